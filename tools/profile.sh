#!/bin/bash
# rocprofv3 kernel-trace summary + PMC passes of bench.py's headline leg (GPU box).
# Output: gpurun_out/prof_<tag>/
#  trace/      --kernel-trace --stats of the driver's bench command (--steps 20 --warmup 5), headline
#              leg only, so the averages are config-2 launches; bench.json = that run's own line
#  pmc_*/      one counter pass per run (counter-block limits: 8 SQ, 4 TCC (FETCH_SIZE uses 3), 2 GRBM)
set -o pipefail
TAG=${1:-r03}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e"
BENCH="$PWD/bench.py --steps 20 --warmup 5 $LEGS"
PBENCH="$PWD/bench.py --steps 3 --warmup 1 $LEGS"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/bench.json 2> $OUT/trace.log || { tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $PBENCH > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $PBENCH > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_valu -o run -- python3 $PBENCH > $OUT/pmc_valu.log 2>&1 || { tail -20 $OUT/pmc_valu.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --output-format csv -d $OUT/pmc_stall -o run -- python3 $PBENCH > $OUT/pmc_stall.log 2>&1 || { tail -20 $OUT/pmc_stall.log; exit 1; }
find $OUT -name "*.csv" | head -50
