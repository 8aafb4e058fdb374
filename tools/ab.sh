#!/bin/bash
# A/B of lib/variants builds against the default lib on one GPU box: parity of the default build,
# then alternating short benches (default, variant, default, variant) so box drift cancels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/ab_parity.log 2>&1 || { tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -1 gpurun_out/ab_parity.log
for round in 1 2; do
  for v in default "$@"; do
    LIB=""; [ $v != default ] && LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so
    HLC_LIB=$LIB timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$round $v', round(d['value']), 'votes/s rec_ms', round(d['roofline']['kernel_ms_avg'],3))"
  done
done
