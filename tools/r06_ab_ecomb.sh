#!/bin/bash
# Round-6 A/B: the u1 G comb split off the recovery finish and enqueued behind the prehash and the prep
# stage, so that it runs in k_rec_main's tail (HLC_EARLY_COMB=1: k_rec_ucomb + k_rec_add), against the
# fused k_rec_comb after k_rec_main.  Parity first (tests/test_gpu_early_comb.py), then the headline leg,
# 3 alternating rounds, then one traced step of each arm (kernel timeline).
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_gpu_early_comb.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06/early_comb_tests.txt 2>&1 || { tail -30 gpurun_out/r06/early_comb_tests.txt; exit 1; }
tail -2 gpurun_out/r06/early_comb_tests.txt
bash tools/ab_arms.sh ecomb=HLC_EARLY_COMB=1 ecomb2=HLC_EARLY_COMB=2 > gpurun_out/r06/ab_ecomb_headline.txt 2>&1 || { tail gpurun_out/r06/ab_ecomb_headline.txt; exit 1; }
cat gpurun_out/r06/ab_ecomb_headline.txt
cd /tmp && export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
for arm in 0 2; do
  HLC_EARLY_COMB=$arm timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06/ecomb_trace$arm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 $LEGS > $GRAFT_REPO_ROOT/gpurun_out/r06/ecomb_trace$arm.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06/ecomb_trace$arm.log || { tail $GRAFT_REPO_ROOT/gpurun_out/r06/ecomb_trace$arm.log; exit 1; }
done
echo ecomb-done
