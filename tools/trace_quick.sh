#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (GPU box). Output: gpurun_out/trace_<tag>/
set -o pipefail
TAG=${1:-q}
OUT=$PWD/gpurun_out/trace_$TAG
mkdir -p $OUT
BENCH="$PWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config3 --no-wire --no-stream"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:10.1f} total_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
