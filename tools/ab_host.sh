#!/bin/bash
# A/B of library variants on the host-buffer entry: tools/host_pipe.py (default schedule, 8 host
# threads) per arm, arms alternating for 3 rounds.  Arms as in tools/ab_arms.sh (NAME = lib/variants).
set -o pipefail
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in default "$@"; do
    ENVS=""
    [ "$v" != default ] && ENVS="HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so"
    env $ENVS timeout -k 10 200 python tools/host_pipe.py --threads 8 --steps 20 > gpurun_out/abh_$v.txt 2> gpurun_out/abh_$v.err || { tail gpurun_out/abh_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abh_$v.txt').read().splitlines()[-1]);print('$round $v host', round(d['votes_per_s']), 'votes/s', round(d['ms_per_call'],3), 'ms')"
  done
done
