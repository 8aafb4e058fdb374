#!/bin/bash
# Round-6 A/B: the host-buffer entries' per-range prep / main events bound to the kernel dispatches
# (hipExtLaunchKernelGGL stop events, no marker packets) against the previous commit (ctr).
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_wire_pipeline.py tests/test_gpu_host_fuzz.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e/hostev_tests.txt 2>&1 || { tail -30 gpurun_out/r06e/hostev_tests.txt; exit 1; }
tail -2 gpurun_out/r06e/hostev_tests.txt
AB_MODE=host bash tools/ab_arms.sh ctr > gpurun_out/r06e/ab_hostev_host.txt 2>&1 || { tail gpurun_out/r06e/ab_hostev_host.txt; exit 1; }
cat gpurun_out/r06e/ab_hostev_host.txt
AB_MODE=wire bash tools/ab_arms.sh ctr > gpurun_out/r06e/ab_hostev_wire.txt 2>&1 || { tail gpurun_out/r06e/ab_hostev_wire.txt; exit 1; }
cat gpurun_out/r06e/ab_hostev_wire.txt
