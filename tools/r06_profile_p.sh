#!/bin/bash
# Round-6 profile refresh on the shipped build (the final build: inversion early exit, products mod n over 29-bit limbs, the 24-bit comb in shared
# per-device tables): tools/profile.sh r06p, then the driver's bench command with every leg.
set -o pipefail
mkdir -p gpurun_out/r06p
bash tools/profile.sh r06p > gpurun_out/r06p/profile.log 2>&1 || { tail -30 gpurun_out/r06p/profile.log; exit 1; }
python tools/bench_summary.py gpurun_out/prof_r06p/bench.json
rm -rf profiles/r06p_rocprof && cp -r gpurun_out/prof_r06p profiles/r06p_rocprof  # the bench line below reads roofline.json's profile
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06p/bench_detail.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06p/bench.json 2> gpurun_out/r06p/bench.err || { tail gpurun_out/r06p/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06p/bench.json
