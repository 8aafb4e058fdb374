#!/bin/bash
# Round-6 A/B: the prep stage's work counters cleared by k_red_init (no memset on the aux stream before
# k_rec_prep) against the previous commit's library (kev2); the late chain schedule (HLC_EARLY_COMB=5:
# k_chain_small behind k_rec_main on the least-priority stream); k_rec_final at 4 votes per inversion
# (fin4) and with its loads issued ahead of use (finld) on top of the new build.
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_early_comb.py tests/test_gpu_scenarios.py tests/test_gpu_tally.py tests/test_gpu_options.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e/ctr_tests.txt 2>&1 || { tail -30 gpurun_out/r06e/ctr_tests.txt; exit 1; }
tail -2 gpurun_out/r06e/ctr_tests.txt
bash tools/ab_arms.sh kev2 late=HLC_EARLY_COMB=5 fin4 finld > gpurun_out/r06e/ab_ctr_headline.txt 2>&1 || { tail gpurun_out/r06e/ab_ctr_headline.txt; exit 1; }
cat gpurun_out/r06e/ab_ctr_headline.txt
cd /tmp && export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
HLC_EARLY_COMB=5 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06e/late_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 $LEGS > $GRAFT_REPO_ROOT/gpurun_out/r06e/late_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06e/late_trace.log || { tail $GRAFT_REPO_ROOT/gpurun_out/r06e/late_trace.log; exit 1; }
echo late-done
