#!/bin/bash
# Round-6 profile refresh on the shipped schedule (digit prefetch, early comb): the per-call fixed cost of
# this box (tools/size_sweep.py: 160k .. 5.1M votes per call), then tools/profile.sh r06b.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u tools/size_sweep.py 2500 5000 10000 20000 40000 80000 > gpurun_out/r06/size_sweep_b.txt 2>&1 || { tail gpurun_out/r06/size_sweep_b.txt; exit 1; }
cat gpurun_out/r06/size_sweep_b.txt
bash tools/profile.sh r06b > gpurun_out/r06/profile_b.log 2>&1 || { tail -30 gpurun_out/r06/profile_b.log; exit 1; }
python tools/bench_summary.py gpurun_out/prof_r06b/bench.json
