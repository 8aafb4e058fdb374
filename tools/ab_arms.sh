#!/bin/bash
# A/B over named arms, arms alternating for 3 rounds on one box.
#   bash tools/ab_arms.sh ARM [ARM ...]           (the shipped library runs as arm "default" first)
# An arm is NAME or NAME=ENV...: NAME alone loads lib/variants/libhlc_NAME.so (make variant NAME=...);
# NAME=ENV runs the shipped lib under that env (e.g. one=HLC_SPLIT_VOTES=0).  Names starting with
# probe/nofence/norel mark timing probes (HLC_BENCH_PROBE=1 skips bench.py's outcome guard).
# AB_MODE selects what each arm runs:
#   headline (default)  bench.py headline leg, 150 timed steps after 50 warm-up
#   legs                bench.py headline + config-5 legs, 20 steps
#   c4                  bench.py headline (3 steps) + the config-4 shard leg (12.5M votes per call)
#   host                tools/host_pipe.py (host-buffer entry, default schedule, 8 host threads), 20 calls
#   wire                tools/wire_pipe.py (the wire entry from host buffers, default schedule), 20 calls
#                       (AB_WIRE_ARGS="--device-walk lane" adds the device-resident wire entry)
#                       (host_pipe.py sets HLC_SPLIT_VOTES / HLC_HOST_THREADS itself: vary those with its flags)
set -o pipefail
mkdir -p gpurun_out
MODE=${AB_MODE:-headline}
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
for round in 1 2 3; do
  for arm in default "$@"; do
    v=${arm%%=*}; ENVS=""
    if [ "$arm" != "$v" ]; then ENVS="${arm#*=}"
    elif [ "$v" != default ]; then ENVS="HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so"; fi
    case $v in probe*|nofence*|norel*) ENVS="$ENVS HLC_BENCH_PROBE=1";; esac
    O=gpurun_out/ab_${MODE}_$v
    case $MODE in
    headline)
      HLC_BENCH_DETAIL=$PWD/$O.detail.json env $ENVS timeout -k 10 200 python bench.py --steps 150 --warmup 50 $LEGS > $O.json 2> $O.err || { tail $O.err; exit 1; }
      python -c "import json;d=json.load(open('$O.json'));print('$round $v', round(d['value']), 'votes/s rec_ms', round(d['roofline']['kernel_ms_avg'],3), 'step_ms', round(d['ms_per_step'],3), 'GHz', d['roofline'].get('live_k_rec_main_GHz'))" ;;
    legs)
      HLC_BENCH_DETAIL=$PWD/$O.detail.json env $ENVS timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${LEGS/--no-config5/} > $O.json 2> $O.err || { tail $O.err; exit 1; }
      python -c "import json;d=json.load(open('$O.json'));print('$round $v headline', round(d['value']), 'config5', round(d['legs']['config5']), 'votes/s')" ;;
    c4)
      HLC_BENCH_DETAIL=$PWD/$O.detail.json env $ENVS timeout -k 10 300 python bench.py --steps 3 --warmup 1 ${LEGS/--no-config4-shard/} > $O.json 2> $O.err || { tail $O.err; exit 1; }
      python -c "import json;d=json.load(open('$O.json'));print('$round $v config4_shard', round(d['legs']['config4_shard']), 'votes/s headline', round(d['value']))" ;;
    host)
      env $ENVS timeout -k 10 200 python tools/host_pipe.py --threads 8 --steps 20 > $O.txt 2> $O.err || { tail $O.err; exit 1; }
      python -c "import json;d=json.loads(open('$O.txt').read().splitlines()[-1]);print('$round $v host', round(d['votes_per_s']), 'votes/s', round(d['ms_per_call'],3), 'ms')" ;;
    wire)
      env $ENVS timeout -k 10 200 python tools/wire_pipe.py --steps 20 $AB_WIRE_ARGS > $O.txt 2> $O.err || { tail $O.err; exit 1; }
      python -c "
import json
for l in open('$O.txt'):
    d=json.loads(l); print('$round $v wire', d.get('device_resident_walk', 'from-host'), round(d['votes_per_s']), 'votes/s', round(d['ms_per_call'],3), 'ms')" ;;
    *)
      echo "unknown AB_MODE $MODE"; exit 2 ;;
    esac
  done
done
