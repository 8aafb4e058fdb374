#!/bin/bash
# One GPU-box session as a list of steps, run in order; the first failing step ends the call.
#   bash tools/gpu.sh TAG step [step ...]          (outputs under gpurun_out/, named by TAG)
# Steps:
#   tests      the whole -m gpu suite (one process, per-test timeouts)
#   quick      parity subset (test_gpu_parity + test_gpu_scenarios, no config 3)
#   ptest      pytest $PTEST -m gpu (a subset of the suite)
#   smoke      __graft_entry__.smoke()
#   bench      the driver's command: bench.py --gpus 1 --steps 20 --warmup 5 (every leg)
#   qbench     headline leg only, 5 steps
#   n2         N = 2 dry run of the sharded bench (gloo, both ranks on GPU 0): config-4 shards
#   rccl1      the N > 1 bench path at one rank over RCCL (HLC_BENCH_DIST=1): config-4 shard, exchange on GPU
#   pipe       tools/host_pipe.py sweep, arguments from $PIPE_ARGS
#   wirepipe   tools/wire_pipe.py sweep (the wire entry from host buffers), arguments from $WIRE_ARGS
#   fetchcalib tools/fetch_calib under rocprofv3 FETCH_SIZE / WRITE_SIZE passes: counter bytes per access shape
#   counters   rocprofv3 -L on the box; tools/fetch_calib under the L2 request-size counters when present
#   teardownprof  tools/host_pipe.py under rocprofv3 --kernel-trace --stats: exit status must be 0
#   pipetrace  rocprofv3 kernel + memory-copy trace of one host-buffer setting ($PIPE_ARGS)
#   verify     tools/verify_latency.py (hlc_eth_verify_batch at the C ABI)
#   profile    tools/profile.sh TAG (kernel trace + PMC passes of the headline leg)
#   ab         tools/ab_arms.sh $AB_ARMS (alternating A/B arms: lib/variants builds or env settings;
#              $AB_MODE = headline / legs / host)
#   clock      tools/clock_probe.py (the library's k_rec_main clock stamps), two rounds; $CLOCK_VARIANTS names
#              lib/variants/libhlc_NAME.so builds to alternate with the shipped library ("shipped")
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
O=gpurun_out
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e"
fail() { echo "step $1 failed"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 200 --timeout-method thread \
      > $O/gpu_tests_$TAG.log 2>&1 || fail tests $O/gpu_tests_$TAG.log
    tail -2 $O/gpu_tests_$TAG.log ;;
  quick)
    timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "not config3" > $O/quick_$TAG.log 2>&1 || fail quick $O/quick_$TAG.log
    tail -1 $O/quick_$TAG.log ;;
  ptest)
    timeout -k 10 600 python -u -m pytest $PTEST -m gpu -x -v --timeout 200 --timeout-method thread \
      > $O/ptest_$TAG.log 2>&1 || fail ptest $O/ptest_$TAG.log
    tail -2 $O/ptest_$TAG.log ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || fail smoke $O/smoke_$TAG.log
    tail -1 $O/smoke_$TAG.log ;;
  bench)
    timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$TAG.json 2> $O/bench_$TAG.err || fail bench $O/bench_$TAG.err
    python tools/bench_summary.py $O/bench_$TAG.json ;;
  qbench)
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 $LEGS > $O/qbench_$TAG.json 2> $O/qbench_$TAG.err || fail qbench $O/qbench_$TAG.err
    python tools/bench_summary.py $O/qbench_$TAG.json ;;
  n2)
    HLC_BENCH_BACKEND=gloo HLC_BENCH_SAME_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 4 --proposals 20000 \
      --steps 5 --warmup 2 > $O/n2_$TAG.json 2> $O/n2_$TAG.err || fail n2 $O/n2_$TAG.err
    python tools/bench_summary.py $O/n2_$TAG.json ;;
  rccl1)
    HLC_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --config 4 --proposals 20000 --steps 5 --warmup 2 \
      $LEGS > $O/rccl1_$TAG.json 2> $O/rccl1_$TAG.err || fail rccl1 $O/rccl1_$TAG.err
    python tools/bench_summary.py $O/rccl1_$TAG.json ;;
  pipe)
    timeout -k 10 500 python tools/host_pipe.py $PIPE_ARGS > $O/pipe_$TAG.txt 2> $O/pipe_$TAG.err || fail pipe $O/pipe_$TAG.err
    cat $O/pipe_$TAG.txt ;;
  wirepipe)
    timeout -k 10 500 python tools/wire_pipe.py $WIRE_ARGS > $O/wirepipe_$TAG.txt 2> $O/wirepipe_$TAG.err || fail wirepipe $O/wirepipe_$TAG.err
    cat $O/wirepipe_$TAG.txt ;;
  fetchcalib)
    OUT=$PWD/$O/fetchcalib_$TAG
    mkdir -p $OUT
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 $OLDPWD/tools/fetch_calib > $OUT/plain.txt 2>&1 && \
      timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $OLDPWD/tools/fetch_calib \
        > $OUT/fetch.txt 2>&1 && \
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $OLDPWD/tools/fetch_calib \
        > $OUT/write.txt 2>&1) || fail fetchcalib $OUT/fetch.txt
    python tools/fetch_calib.py $OUT/fetch $OUT/write $OUT/plain.txt | tee $OUT/summary.json ;;
  counters)
    # the counters this rocprofv3 offers on the box, then (when it has them) tools/fetch_calib under the L2's
    # request-size counters: which shapes issue 128-B requests that FETCH_SIZE tallies at 64 B
    OUT=$PWD/$O/counters_$TAG
    mkdir -p $OUT
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1) || true
    grep -o "TCC_[A-Z0-9_]*" $OUT/list.txt | sort -u > $OUT/tcc.txt || true
    if grep -qx "TCC_EA0_RDREQ_128B" $OUT/tcc.txt && grep -qx "TCC_EA0_RDREQ" $OUT/tcc.txt; then
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B \
        TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_32B --output-format csv -d $OUT/req -o run -- $OLDPWD/tools/fetch_calib \
        > $OUT/req.txt 2>&1) || echo "request-size pass failed"
    fi
    wc -l $OUT/tcc.txt ;;
  teardownprof)
    # the host pipeline tool under rocprofv3 must exit 0 (no SIGSEGV in the finalizers)
    OUT=$PWD/$O/teardown_$TAG
    mkdir -p $OUT
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT \
      -o run -- python3 $OLDPWD/tools/host_pipe.py --steps 3 > $OUT/out.txt 2> $OUT/err.txt; echo "exit $?" > $OUT/rc.txt)
    cat $OUT/rc.txt; grep -q "exit 0" $OUT/rc.txt || fail teardownprof $OUT/err.txt ;;
  pipetrace)
    OUT=$PWD/$O/pipetrace_$TAG
    mkdir -p $OUT
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $OUT -o run -- python3 $OLDPWD/tools/host_pipe.py $PIPE_ARGS > $OUT/out.txt 2> $OUT/err.txt) \
      || fail pipetrace $OUT/err.txt
    cat $OUT/out.txt ;;
  verify)
    timeout -k 10 400 python tools/verify_latency.py $VERIFY_ARGS > $O/verify_$TAG.txt 2> $O/verify_$TAG.err || fail verify $O/verify_$TAG.err
    cat $O/verify_$TAG.txt ;;
  profile)
    bash tools/profile.sh $TAG || exit 1 ;;
  ab)
    bash tools/ab_arms.sh $AB_ARMS || exit 1 ;;
  clock)
    for round in 1 2; do
      for v in shipped $CLOCK_VARIANTS; do
        L=""; [ $v != shipped ] && L=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so
        HLC_LIB=$L timeout -k 10 200 python tools/clock_probe.py \
          run --tag $v > $O/clock_${TAG}_${v}_$round.log 2>&1 || fail clock $O/clock_${TAG}_${v}_$round.log
      done
    done
    python tools/clock_probe.py summarize $O/clock_${TAG}_*.log | tee $O/clock_$TAG.txt ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
