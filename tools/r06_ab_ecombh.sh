#!/bin/bash
# Round-6 A/B: early comb for the host-buffer entries (HLC_EARLY_COMB=3: bit 2 adds k_rec_ucomb behind every
# recovery range's prep stage) against the device-only default (1): the SoA host entry (tools/host_pipe.py)
# and the pipelined wire entry (tools/wire_pipe.py), 3 alternating rounds each; parity first.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_gpu_early_comb.py tests/test_gpu_options.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06/early_comb_host_tests.txt 2>&1 || { tail -30 gpurun_out/r06/early_comb_host_tests.txt; exit 1; }
tail -2 gpurun_out/r06/early_comb_host_tests.txt
AB_MODE=host bash tools/ab_arms.sh ecombh=HLC_EARLY_COMB=3 > gpurun_out/r06/ab_ecombh_host.txt 2>&1 || { tail gpurun_out/r06/ab_ecombh_host.txt; exit 1; }
cat gpurun_out/r06/ab_ecombh_host.txt
AB_MODE=wire bash tools/ab_arms.sh ecombh=HLC_EARLY_COMB=3 > gpurun_out/r06/ab_ecombh_wire.txt 2>&1 || { tail gpurun_out/r06/ab_ecombh_wire.txt; exit 1; }
cat gpurun_out/r06/ab_ecombh_wire.txt
