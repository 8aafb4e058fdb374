#!/bin/bash
# A/B of library variants on the bench line's headline and config-5 legs (20 steps, arms alternating,
# 3 rounds).  Arms as in tools/ab_arms.sh (NAME = lib/variants/libhlc_NAME.so).
set -o pipefail
mkdir -p gpurun_out
LEGS="--no-cpu-baseline --no-config3 --no-wire --no-stream --no-e2e"
for round in 1 2 3; do
  for v in default "$@"; do
    ENVS=""
    [ "$v" != default ] && ENVS="HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so"
    env $ENVS timeout -k 10 300 python bench.py --steps 20 --warmup 5 $LEGS > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { tail gpurun_out/abl_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abl_$v.json'));print('$round $v headline', round(d['value']), 'config5', round(d['config5']['value']), 'votes/s')"
  done
done
