#!/bin/bash
# Round 3, third GPU call: host pipeline, device config-5 leg, glds / table-sharing A/B, verify latency.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_config5_device.py tests/test_gpu_tally.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03c_new.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03c_new.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03c_new.log
timeout -k 10 300 python tools/host_pipe.py --steps 10 --chunks 0,65536,131072,262144 > gpurun_out/host_pipe_r03c.txt 2>&1 || { tail -20 gpurun_out/host_pipe_r03c.txt; exit 1; }
grep chunk_votes gpurun_out/host_pipe_r03c.txt
timeout -k 10 300 python tools/verify_latency.py --sizes 1,8,64,1024,65536 > gpurun_out/verify_latency_r03c.txt 2>&1 || { tail -20 gpurun_out/verify_latency_r03c.txt; exit 1; }
grep '"n"' gpurun_out/verify_latency_r03c.txt
bash tools/ab_long.sh glds probe_share2 probe_share64 > gpurun_out/ab_r03c.txt 2>&1 || { tail -20 gpurun_out/ab_r03c.txt; exit 1; }
cat gpurun_out/ab_r03c.txt | grep votes
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03c.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r03c.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03c.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || { tail -20 gpurun_out/bench_r03c.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r03c.json'));print('bench', round(d['value']), 'ms', round(d['ms_per_step'],3), 'e2e', round(d['end_to_end']['value']), 'c5', round(d['config5']['value']), 'cpu', round(d['cpu_baseline']['value']), 'x', round(d['gpu_over_cpu']))"
