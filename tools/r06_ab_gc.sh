#!/bin/bash
# Round-6 call: (1) A/B of wider u1 G comb windows now that the comb runs after k_rec_main (k_rec_ucomb):
# W = 24 (11 additions, 5.9 GB table) and W = 26 (10 additions, 21.5 GB) against the shipped W = 22 (12,
# 1.5 GB), parity of the W = 26 build first; (2) the committed profile refreshed on the shipped build
# (tools/profile.sh r06h) and the driver's bench command with every leg.
set -o pipefail
mkdir -p gpurun_out/r06h
HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_gc26.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h/tests_gc26.txt 2>&1 || { tail -30 gpurun_out/r06h/tests_gc26.txt; exit 1; }
tail -1 gpurun_out/r06h/tests_gc26.txt
bash tools/ab_arms.sh gc24 gc26 > gpurun_out/r06h/ab_gc.txt 2>&1 || { tail gpurun_out/r06h/ab_gc.txt; exit 1; }
cat gpurun_out/r06h/ab_gc.txt
bash tools/profile.sh r06h > gpurun_out/r06h/profile.log 2>&1 || { tail -30 gpurun_out/r06h/profile.log; exit 1; }
python tools/bench_summary.py gpurun_out/prof_r06h/bench.json
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06h/bench_detail.json timeout -k 10 300 python bench.py > gpurun_out/r06h/bench.json 2> gpurun_out/r06h/bench.err || { tail gpurun_out/r06h/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06h/bench.json
