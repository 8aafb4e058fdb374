#!/bin/bash
# Quick GPU iteration: parity subset + bench without CPU baseline. Output: gpurun_out/
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not config3" > gpurun_out/quick_$TAG.log 2>&1 || { tail -30 gpurun_out/quick_$TAG.log; exit 1; }
tail -2 gpurun_out/quick_$TAG.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('$TAG', round(d['value']), 'votes/s', 'rec_ms', round(d['roofline']['kernel_ms_avg'],3), 'frac', round(d['roofline']['frac'],3))"
