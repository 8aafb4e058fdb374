#!/bin/bash
# Round-6 A/B: k_rec_final with every vote's loads issued ahead (HLC_FIN_LOADS=1) at 8, 10 and 12 votes per
# lane (10: 64,000 lanes, at most one wave per SIMD) against the shipped build (8 votes, loads in turn).
# Parity of the 10-vote arm first.
set -o pipefail
mkdir -p gpurun_out/r06m
HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_fin10L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m/tests_fin10L.txt 2>&1 || { tail -30 gpurun_out/r06m/tests_fin10L.txt; exit 1; }
tail -1 gpurun_out/r06m/tests_fin10L.txt
bash tools/ab_arms.sh fin8L fin10L fin12L > gpurun_out/r06m/ab_finl.txt 2>&1 || { tail gpurun_out/r06m/ab_finl.txt; exit 1; }
cat gpurun_out/r06m/ab_finl.txt
