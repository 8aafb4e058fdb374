#!/bin/bash
# One GPU call: gpu tests, smoke, bench (with cpu baseline), rocprof kernel-trace summary. Output: gpurun_out/
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash tools/profile.sh $TAG
