#!/bin/bash
# Round-6 call: the vote statuses written by k_rec_addr (no k_vote_status launch) and the large-proposal
# chain check behind the tables on the aux stream (early comb) -- the whole GPU suite on that build and
# smoke(), then A/B against the round-6 head library (lib/variants/libhlc_r6g.so) and the votes-per-lane
# arms of k_rec_final (FIN_BATCH) / k_rec_prep (REC_BATCH): 10 votes per lane makes 64,000 lanes for 640k
# votes, one wave per SIMD (8 per lane: 1,250 waves, two on some SIMDs).
set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06f/gpu_all.txt 2>&1 || { tail -30 gpurun_out/r06f/gpu_all.txt; exit 1; }
tail -1 gpurun_out/r06f/gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06f/smoke.txt 2>&1 || { tail -20 gpurun_out/r06f/smoke.txt; exit 1; }
tail -1 gpurun_out/r06f/smoke.txt
for v in fin10 both10; do
  HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_early_comb.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f/tests_$v.txt 2>&1 || { tail -30 gpurun_out/r06f/tests_$v.txt; exit 1; }
  tail -1 gpurun_out/r06f/tests_$v.txt
done
bash tools/ab_arms.sh r6g fin10 both10 fin16 prep10 > gpurun_out/r06f/ab_fin.txt 2>&1 || { tail gpurun_out/r06f/ab_fin.txt; exit 1; }
cat gpurun_out/r06f/ab_fin.txt
