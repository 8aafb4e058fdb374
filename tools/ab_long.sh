#!/bin/bash
# A/B of lib/variants builds against the default lib on one GPU box, at steady-state power: each
# arm runs the headline leg for --steps 150 after 50 warm-up steps (~1.4 s back to back), arms
# alternate for 3 rounds so box drift cancels.  Usage: bash tools/ab_long.sh variant...
# Variants named probe* are timing probes with wrong results (HLC_BENCH_PROBE=1 skips the guard).
set -o pipefail
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in default "$@"; do
    LIB=""; [ $v != default ] && LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so
    PROBE=0; case $v in probe*) PROBE=1;; esac
    HLC_BENCH_PROBE=$PROBE HLC_LIB=$LIB timeout -k 10 200 python bench.py --steps 150 --warmup 50 --no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { tail gpurun_out/abl_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abl_$v.json'));print('$round $v', round(d['value']), 'votes/s rec_ms', round(d['roofline']['kernel_ms_avg'],3), 'step_ms', round(d['ms_per_step'],3))"
  done
done
