#!/bin/bash
# Round-6 A/B: k_rec_ucomb forms Q itself for every vote whose u2 R k_rec_main has published
# (HLC_UCOMB_ADD=1, the default build) against the same build without it (lib/variants/libhlc_noadd.so)
# and the round-6 head library (libhlc_r6g.so).  Parity first, then the headline leg (3 alternating
# rounds), then one kernel trace of the default build for the step timeline.
set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 700 python -u -m pytest tests/test_gpu_early_comb.py tests/test_gpu_scenarios.py tests/test_gpu_parity.py tests/test_gpu_exact_chains.py tests/test_gpu_options.py tests/test_gpu_host_pipeline.py tests/test_gpu_config5_device.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06g/uadd_tests.txt 2>&1 || { tail -30 gpurun_out/r06g/uadd_tests.txt; exit 1; }
tail -1 gpurun_out/r06g/uadd_tests.txt
bash tools/ab_arms.sh noadd r6g > gpurun_out/r06g/ab_uadd.txt 2>&1 || { tail gpurun_out/r06g/ab_uadd.txt; exit 1; }
cat gpurun_out/r06g/ab_uadd.txt
cd /tmp && export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-config3 --no-config5 --no-wire --no-stream --no-e2e --no-config4-shard"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06g/uadd_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 $LEGS > $GRAFT_REPO_ROOT/gpurun_out/r06g/uadd_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06g/uadd_trace.log || { tail $GRAFT_REPO_ROOT/gpurun_out/r06g/uadd_trace.log; exit 1; }
echo trace-done
