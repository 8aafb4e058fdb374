#!/bin/bash
# Round-6 A/B: timing events bound to kernel dispatches (hipExtLaunchKernelGGL), the fork / prep / join
# events bound the same way, the flag word cleared by k_red_init, and the large-proposal tables behind
# k_rec_main on the aux stream -- against the round-6 library before them (lib/variants/libhlc_r6base.so).
# Probe first, then parity, then the headline leg (3 alternating rounds), then one traced run.
set -o pipefail
mkdir -p gpurun_out/r06e
true
true
timeout -k 10 600 python -u -m pytest tests/test_gpu_early_comb.py tests/test_gpu_scenarios.py tests/test_gpu_tally.py tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_host_pipeline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e/kev2_tests.txt 2>&1 || { tail -30 gpurun_out/r06e/kev2_tests.txt; exit 1; }
tail -2 gpurun_out/r06e/kev2_tests.txt
bash tools/ab_arms.sh r6base > gpurun_out/r06e/ab_kev2_headline.txt 2>&1 || { tail gpurun_out/r06e/ab_kev2_headline.txt; exit 1; }
cat gpurun_out/r06e/ab_kev2_headline.txt
cd /tmp && export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06e/kev2_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 $LEGS > $GRAFT_REPO_ROOT/gpurun_out/r06e/kev2_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06e/kev2_trace.log || { tail $GRAFT_REPO_ROOT/gpurun_out/r06e/kev2_trace.log; exit 1; }
echo kev-done
