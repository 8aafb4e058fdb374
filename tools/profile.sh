#!/bin/bash
# rocprofv3 kernel traces + PMC passes behind bench.py's roofline and chain/tally figures (GPU box).
# Output: gpurun_out/prof_<tag>/ (copied to profiles/<round>_rocprof/ and named in roofline.json)
#  trace/          --kernel-trace --stats of the driver's bench command (--steps 20 --warmup 5), headline
#                  leg only, so the averages are config-2 launches; bench.json = that run's own line
#  trace_serial/   the same with HLC_SERIAL_STAGES=1 (every kernel alone on one stream): isolated
#                  durations of the chain / tally kernels
#  pmc_*/          one counter pass per run (counter-block limits: 8 SQ, 4 TCC (FETCH_SIZE uses 3), 2 GRBM);
#                  pmc_req: the L2 read requests by size (TCC_EA0_RDREQ, _128B, _32B) for exact read bytes
#  c3_trace/, c3_fetch/, c3_write/, c3_req/   config 3 (tools/config3_time.py: 1 proposal, 1M chained votes)
set -o pipefail
TAG=${1:-r04}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
BENCH="$PWD/bench.py --steps 20 --warmup 5 $LEGS"
PBENCH="$PWD/bench.py --steps 3 --warmup 1 $LEGS"
C3="$PWD/tools/config3_time.py 3"
cd /tmp && export TMPDIR=/tmp
run() {  # run NAME LIMIT rocprofv3-args... -- program...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 -s KILL $lim rocprofv3 "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/bench.json 2> $OUT/trace.log || { tail -20 $OUT/trace.log; exit 1; }
HLC_SERIAL_STAGES=1 run trace_serial 300 --kernel-trace --stats --output-format csv -d $OUT/trace_serial -o run -- python3 $PBENCH
run pmc_fetch 300 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $PBENCH
run pmc_write 300 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $PBENCH
# the L2's read requests by size (bench.py read_bytes: FETCH_SIZE tallies 128-B requests at 64 B on gfx950)
run pmc_req 300 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B --output-format csv -d $OUT/pmc_req -o run -- python3 $PBENCH
run pmc_valu 300 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_valu -o run -- python3 $PBENCH
run pmc_stall 300 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --output-format csv -d $OUT/pmc_stall -o run -- python3 $PBENCH
run c3_trace 300 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o run -- python3 $C3
run c3_fetch 300 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/c3_fetch -o run -- python3 $C3
run c3_write 300 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/c3_write -o run -- python3 $C3
run c3_req 300 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B --output-format csv -d $OUT/c3_req -o run -- python3 $C3
find $OUT -name "*.csv" | head -60
