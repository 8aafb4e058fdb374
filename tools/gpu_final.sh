#!/bin/bash
# Final verification of the shipped build: the whole GPU suite, smoke, the driver's bench command,
# then the committed profile (kernel trace + PMC passes) of the same command.  Output: gpurun_out/
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', round(d['value']), 'ms', round(d['ms_per_step'],3), 'e2e', round(d['end_to_end']['value']), 'c5', round(d['config5']['value']), 'cpu', round(d['cpu_baseline']['value']))"
bash tools/profile.sh $TAG
