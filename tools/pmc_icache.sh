#!/bin/bash
# Instruction-cache / instruction-wait PMC pass over a short bench (GPU box), per HLC_LIB variant.
set -o pipefail
for v in ${@:-default}; do
  OUT=$PWD/gpurun_out/pmc_icache_$v
  mkdir -p $OUT
  LIB=""
  [ $v != default ] && LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so
  BENCH="$PWD/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-wire --no-stream"
  ( cd /tmp && export TMPDIR=/tmp && HLC_LIB=$LIB timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d $OUT -o run -- python3 $BENCH > $OUT/pmc.log 2>&1 ) || { tail -20 $OUT/pmc.log; exit 1; }
  f=$(find $OUT -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "k_rec_main" in k:
        print(sys.argv[2], k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
done
