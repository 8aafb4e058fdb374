#!/bin/bash
# Round-6 call: the 24-bit u1 G comb (11 additions, 5.9 GB) in per-device tables shared by the contexts --
# context-creation cost and memory, the whole GPU suite and smoke() on it, then the headline A/B against
# the previous build (W = 22, a table per context: lib/variants/libhlc_r6h.so), 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 120 python -u tools/ctx_tables.py > gpurun_out/r06i/ctx_tables.txt 2>&1 || { tail -20 gpurun_out/r06i/ctx_tables.txt; exit 1; }
cat gpurun_out/r06i/ctx_tables.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06i/gpu_all.txt 2>&1 || { tail -30 gpurun_out/r06i/gpu_all.txt; exit 1; }
tail -1 gpurun_out/r06i/gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06i/smoke.txt 2>&1 || { tail -20 gpurun_out/r06i/smoke.txt; exit 1; }
tail -1 gpurun_out/r06i/smoke.txt
bash tools/ab_arms.sh r6h > gpurun_out/r06i/ab_gc24.txt 2>&1 || { tail gpurun_out/r06i/ab_gc24.txt; exit 1; }
cat gpurun_out/r06i/ab_gc24.txt
