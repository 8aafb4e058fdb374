#!/bin/bash
# Round-3 first GPU call: GPU tests, smoke, the driver's bench command, the clock investigation
# (k_rec_main alone / table traffic kept in L1-L2 / hot gathers / the point-op
# loop at the kernel's occupancy), and the rocprof profile of the headline leg.  Output: gpurun_out/
set -o pipefail
mkdir -p gpurun_out
V=$PWD/hashgraph-like-consensus_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r03a.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r03a.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03a.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03a.log 2>&1 || { tail -20 gpurun_out/smoke_r03a.log; exit 1; }
tail -1 gpurun_out/smoke_r03a.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || { tail -20 gpurun_out/bench_r03a.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r03a.json'));print('bench', round(d['value']), 'ms', round(d['ms_per_step'],3), 'e2e', round(d['end_to_end']['value']), 'cpu', round(d['cpu_baseline']['value']))"
for v in clk:0 clk:1 clkwt:0 clkhot:0; do
  n=${v%%:*}; ser=${v##*:}
  HLC_LIB=$V/libhlc_$n.so HLC_SERIAL_STAGES=$ser timeout -k 10 120 python tools/clock_probe.py run --tag ${n}_s$ser > gpurun_out/clk_${n}_s$ser.log 2>&1 || { tail -5 gpurun_out/clk_${n}_s$ser.log; exit 1; }
done
python tools/clock_probe.py summarize gpurun_out/clk_*_s*.log
for m in "rand 3" "same 3" "rand 4" "rand 2"; do
  timeout -k 10 60 ./tools/clock_ubench $m 3 || exit 1
done
bash tools/profile.sh r03a || exit 1
python tools/kstats.py gpurun_out/prof_r03a/trace
