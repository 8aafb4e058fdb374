#!/bin/bash
# Round-6 A/B on the final build: the existing loads-ahead knobs of k_rec_final (HLC_FIN_LOADS=1) and
# k_rec_prep (HLC_PREP_LOADS=1 / 2) and both, against the shipped build.  Parity of the combined arm first.
set -o pipefail
mkdir -p gpurun_out/r06q
HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_allL.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q/tests_allL.txt 2>&1 || { tail -30 gpurun_out/r06q/tests_allL.txt; exit 1; }
tail -1 gpurun_out/r06q/tests_allL.txt
bash tools/ab_arms.sh finL prepL1 prepL2 allL > gpurun_out/r06q/ab_loads.txt 2>&1 || { tail gpurun_out/r06q/ab_loads.txt; exit 1; }
cat gpurun_out/r06q/ab_loads.txt
