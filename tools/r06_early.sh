#!/bin/bash
# Round-6 call: the safegcd inversion stops once g == 0 (18 batches per wave instead of 20): the GPU suite, smoke(),
# then the headline A/B against the same build that always runs 20 batches (lib/variants/libhlc_ct20.so).
set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06o/gpu_all.txt 2>&1 || { tail -30 gpurun_out/r06o/gpu_all.txt; exit 1; }
tail -1 gpurun_out/r06o/gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06o/smoke.txt 2>&1 || { tail -20 gpurun_out/r06o/smoke.txt; exit 1; }
tail -1 gpurun_out/r06o/smoke.txt
bash tools/ab_arms.sh ct20 > gpurun_out/r06o/ab_early.txt 2>&1 || { tail gpurun_out/r06o/ab_early.txt; exit 1; }
cat gpurun_out/r06o/ab_early.txt
