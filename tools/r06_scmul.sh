#!/bin/bash
# Round-6 call: the products mod n over 29-bit limbs (hlc_scmul.hpp; 315 VALU instructions, the 8 x 32 CIOS
# form 732) -- the whole GPU suite and smoke() on it, then the headline A/B against the same build with
# the CIOS form in the recovery kernels (lib/variants/libhlc_cios.so), 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06k/gpu_all.txt 2>&1 || { tail -30 gpurun_out/r06k/gpu_all.txt; exit 1; }
tail -1 gpurun_out/r06k/gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06k/smoke.txt 2>&1 || { tail -20 gpurun_out/r06k/smoke.txt; exit 1; }
tail -1 gpurun_out/r06k/smoke.txt
bash tools/ab_arms.sh cios > gpurun_out/r06k/ab_scmul.txt 2>&1 || { tail gpurun_out/r06k/ab_scmul.txt; exit 1; }
cat gpurun_out/r06k/ab_scmul.txt
