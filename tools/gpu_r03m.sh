#!/bin/bash
# Round 3: k_rec_prep keeps only the batched inversion; u2 / GLV / digits move to k_rec_scalars (one lane per vote).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_exact_chains.py tests/test_gpu_openssl_pin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03m.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03m.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03m.log
bash tools/ab_arms.sh pfused
