#!/bin/bash
# Long A/B over named arms (150 timed steps after 50 warm-up, headline leg, arms alternating for 3
# rounds on one box).  An arm is NAME or NAME=ENV...: NAME alone loads lib/variants/libhlc_NAME.so
# (default: the shipped lib); NAME=ENV runs the shipped lib under that env (e.g. notail=HLC_REC_TAIL=0).
# Names starting with probe/nofence/norel mark timing probes (HLC_BENCH_PROBE=1 skips the guard).
set -o pipefail
mkdir -p gpurun_out
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e"
for round in 1 2 3; do
  for arm in default "$@"; do
    v=${arm%%=*}; ENVS=""
    if [ "$arm" != "$v" ]; then ENVS="${arm#*=}"
    elif [ "$v" != default ]; then ENVS="HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so"; fi
    case $v in probe*|nofence*|norel*) ENVS="$ENVS HLC_BENCH_PROBE=1";; esac
    env $ENVS timeout -k 10 200 python bench.py --steps 150 --warmup 50 $LEGS > gpurun_out/aba_$v.json 2> gpurun_out/aba_$v.err || { tail gpurun_out/aba_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/aba_$v.json'));print('$round $v', round(d['value']), 'votes/s rec_ms', round(d['roofline']['kernel_ms_avg'],3), 'step_ms', round(d['ms_per_step'],3))"
  done
done
