#!/bin/bash
# Round-6 closing call on the final tree: the whole GPU suite, smoke(), and the driver's bench command
# (the committed profile profiles/r06i_rocprof is the one this build was profiled with).
set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06n/gpu_all.txt 2>&1 || { tail -30 gpurun_out/r06n/gpu_all.txt; exit 1; }
tail -1 gpurun_out/r06n/gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06n/smoke.txt 2>&1 || { tail -20 gpurun_out/r06n/smoke.txt; exit 1; }
tail -1 gpurun_out/r06n/smoke.txt
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06n/bench_detail.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06n/bench.json 2> gpurun_out/r06n/bench.err || { tail gpurun_out/r06n/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06n/bench.json
