#!/bin/bash
# Per-arm hardware counters of k_rec_main for a recovery A/B: VALU wave-instructions
# per launch (SQ_INSTS_VALU), bytes written (WRITE_SIZE) and the L2's read requests by size, one rocprofv3
# pass each, over bench.py's headline leg (3 timed steps).  bash tools/ab_pmc.sh ARM [ARM ...]; the shipped
# library runs as arm "default"; ARM loads lib/variants/libhlc_ARM.so.  Output: gpurun_out/abpmc_<arm>/.
set -o pipefail
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
ROOTDIR=$PWD
cd /tmp && export TMPDIR=/tmp
for arm in default "$@"; do
  OUT=$ROOTDIR/gpurun_out/abpmc_$arm
  mkdir -p $OUT
  if [ "$arm" = default ]; then unset HLC_LIB; else export HLC_LIB=$ROOTDIR/hashgraph-like-consensus_amd/lib/variants/libhlc_$arm.so; fi
  export HLC_BENCH_DETAIL=$OUT/detail.json
  for pass in "valu:SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "write:WRITE_SIZE" "req:TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B"; do
    name=${pass%%:*}; ctr=${pass#*:}
    timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/$name -o run -- \
      python3 $ROOTDIR/bench.py --steps 3 --warmup 1 $LEGS > $OUT/$name.json 2> $OUT/$name.log || { tail -20 $OUT/$name.log; exit 1; }
  done
  python3 - "$OUT" "$arm" <<'PY'
import csv, glob, os, sys
out, arm = sys.argv[1], sys.argv[2]
def per_launch(name, counter):
    rows = [r for f in glob.glob(os.path.join(out, name, "**", "*counter_collection.csv"), recursive=True)
            for r in csv.DictReader(open(f)) if "k_rec_main(" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    by = {}
    for r in rows:
        by.setdefault(r["Dispatch_Id"], 0.0)
        by[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(by.values()) / max(len(by), 1), len(by)
V = 640000
valu, k = per_launch("valu", "SQ_INSTS_VALU")
wr, _ = per_launch("write", "WRITE_SIZE")
rd, _ = per_launch("req", "TCC_EA0_RDREQ")
r128, _ = per_launch("req", "TCC_EA0_RDREQ_128B")
r32, _ = per_launch("req", "TCC_EA0_RDREQ_32B")
rbytes = 128 * r128 + 64 * (rd - r128 - r32) + 32 * r32
print(f"{arm}: k_rec_main launches {k}, VALU instructions/vote {valu * 64 / V:.0f} (SQ_INSTS_VALU wave-instructions "
      f"x 64 lanes / votes), read B/vote {rbytes / V:.0f} (L2 read requests by size), write B/vote {wr * 1024 / V:.0f} "
      f"(WRITE_SIZE)")
PY
done
