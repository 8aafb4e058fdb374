#!/bin/bash
# Round-6 profile refresh on the shipped build (vote statuses in k_rec_addr, the 24-bit comb in shared
# per-device tables): tools/profile.sh r06i, then the driver's bench command with every leg.
set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 400 python -u -m pytest tests/test_gpu_tables.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06i/tables_tests.txt 2>&1 || { tail -30 gpurun_out/r06i/tables_tests.txt; exit 1; }
tail -1 gpurun_out/r06i/tables_tests.txt
bash tools/profile.sh r06i > gpurun_out/r06i/profile.log 2>&1 || { tail -30 gpurun_out/r06i/profile.log; exit 1; }
python tools/bench_summary.py gpurun_out/prof_r06i/bench.json
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06i/bench_detail.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06i/bench.json 2> gpurun_out/r06i/bench.err || { tail gpurun_out/r06i/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06i/bench.json
