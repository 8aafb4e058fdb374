#!/bin/bash
# Parity of the default build, then bench every occupancy variant (GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -3 gpurun_out/parity.log
for w in 2 3 4 f32; do
  v=w$w; [ $w = f32 ] && v=f32
  HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config3 --no-wire --no-stream > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err || { tail gpurun_out/bench_w$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_w$w.json'));print('w$w', round(d['value']), 'votes/s', 'rec_ms', round(d['roofline']['kernel_ms_avg'],2), 'frac', round(d['roofline']['frac'],3))"
done
