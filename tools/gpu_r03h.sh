#!/bin/bash
# Round 3: the doubling's Y3 as one sum of two products (fe29_muladd) at a 3-wave register floor.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_exact_chains.py tests/test_gpu_openssl_pin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03h.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03h.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03h.log
bash tools/ab_arms.sh head dblold
