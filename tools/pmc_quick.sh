#!/bin/bash
# One rocprofv3 PMC pass (VALU instruction counts, wave cycles) over a short bench (GPU box).
set -o pipefail
TAG=${1:-q}
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p $OUT
BENCH="$PWD/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-wire --no-stream"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT -o run -- python3 $BENCH > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
f=$(find $OUT -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "k_rec" not in k and "prehash" not in k:
        continue
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
