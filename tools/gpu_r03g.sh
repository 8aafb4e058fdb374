#!/bin/bash
# Round 3: one-reduction Y3 in the mixed addition (fe29_muladd), comb reorder (k_rec_comb at 3 waves),
# prep-first / aux-priority schedule options; host-buffer pipeline sweep + its copy/kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_exact_chains.py tests/test_gpu_openssl_pin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03g.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03g.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03g.log
HLC_PREP_FIRST=1 HLC_AUX_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_scenarios.py -x -q --timeout 200 --timeout-method thread -k "config2_full or config5_byzantine_full or edge_batches or general_path" > gpurun_out/gpu_tests_r03g_pf.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03g_pf.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03g_pf.log
bash tools/ab_arms.sh head madd2 comb4 prepfirst=HLC_PREP_FIRST=1 "both=HLC_PREP_FIRST=1 HLC_AUX_PRIO=1" || exit 1
timeout -k 10 400 python tools/host_pipe.py --steps 8 --chunks 0,65536,131072,262144 --threads 4,8,16 > gpurun_out/host_pipe_r03g.txt 2>&1 || { tail -20 gpurun_out/host_pipe_r03g.txt; exit 1; }
grep chunk_votes gpurun_out/host_pipe_r03g.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pipe -o run -- python3 $GRAFT_REPO_ROOT/tools/host_pipe.py --steps 3 --chunks 131072 --threads 8 > $GRAFT_REPO_ROOT/gpurun_out/prof_pipe.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_pipe.log; exit 1; }
ls $GRAFT_REPO_ROOT/gpurun_out/prof_pipe
