#!/bin/bash
# Round 3: keccak-f[1600] with v_bitop3_b32 (theta's five-way XOR, chi) and v_alignbit_b32 rotations.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_openssl_pin.py tests/test_gpu_host_pipeline.py tests/test_gpu_wire.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03k.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03k.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03k.log
bash tools/ab_arms.sh head
