#!/bin/bash
# Round 3: SHA-256 compression with v_bitop3_b32 (ch, maj, the three-way XORs of the sigmas).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03l.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03l.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03l.log
bash tools/ab_arms.sh head
