#!/bin/bash
# Round 3, second GPU call: the LDS-DMA staged R-table gathers + the device config-5 mutator.
set -o pipefail
mkdir -p gpurun_out
V=$PWD/hashgraph-like-consensus_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_config5_device.py tests/test_gpu_tally.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03b_new.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03b_new.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03b_new.log
bash tools/ab_long.sh noglds share2 || exit 1
for n in clk clknoglds clkshare2; do
  HLC_LIB=$V/libhlc_$n.so timeout -k 10 120 python tools/clock_probe.py run --tag $n > gpurun_out/clkb_$n.log 2>&1 || { tail -5 gpurun_out/clkb_$n.log; exit 1; }
done
python tools/clock_probe.py summarize gpurun_out/clkb_*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03b.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r03b.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03b.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err || { tail -20 gpurun_out/bench_r03b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r03b.json'));print('bench', round(d['value']), 'ms', round(d['ms_per_step'],3), 'c5', round(d['config5']['value']), d['config5']['proposals_by_status'])"
