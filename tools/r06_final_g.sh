#!/bin/bash
# Round-6 verification call: the whole GPU suite, smoke(), and the driver's bench command (GPU box).
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/gpu_all_g.txt 2>&1 || { tail -30 gpurun_out/r06/gpu_all_g.txt; exit 1; }
tail -3 gpurun_out/r06/gpu_all_g.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06/smoke_g.txt 2>&1 || { tail -20 gpurun_out/r06/smoke_g.txt; exit 1; }
tail -1 gpurun_out/r06/smoke_g.txt
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06/bench_g_detail.json timeout -k 10 300 python bench.py > gpurun_out/r06/bench_g.json 2> gpurun_out/r06/bench_g.err || { tail gpurun_out/r06/bench_g.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06/bench_g.json
