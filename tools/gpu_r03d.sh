#!/bin/bash
# Round 3: the page-locked pipelined host entry + outcome-counter kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_wire.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03d_new.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03d_new.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03d_new.log
timeout -k 10 400 python tools/host_pipe.py --steps 10 --chunks 0,32768,65536,131072 --threads 2,4,8 > gpurun_out/host_pipe_r03d.txt 2>&1 || { tail -20 gpurun_out/host_pipe_r03d.txt; exit 1; }
grep chunk_votes gpurun_out/host_pipe_r03d.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-config3 > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err || { tail -20 gpurun_out/bench_r03d.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r03d.json'));print('bench', round(d['value']), 'ms', round(d['ms_per_step'],3), 'e2e', round(d['end_to_end']['value']), 'c5', round(d['config5']['value']), d['counters_per_step'])"
timeout -k 10 600 bash tools/ab_long.sh prio > gpurun_out/ab_prio_r03d.txt 2>&1 || { tail -20 gpurun_out/ab_prio_r03d.txt; exit 1; }
cat gpurun_out/ab_prio_r03d.txt
