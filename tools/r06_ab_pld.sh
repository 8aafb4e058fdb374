#!/bin/bash
# Round-6 A/B: k_rec_prep's per-vote inputs in three memory round trips (HLC_PREP_LOADS=1,
# lib/variants/libhlc_pld.so) against seven (the shipped build), headline leg, 3 rounds; this box's size sweep.
set -o pipefail
mkdir -p gpurun_out/r06
bash tools/ab_arms.sh pld > gpurun_out/r06/ab_pld_headline.txt 2>&1 || { tail gpurun_out/r06/ab_pld_headline.txt; exit 1; }
cat gpurun_out/r06/ab_pld_headline.txt
timeout -k 10 300 python -u tools/size_sweep.py 2500 10000 40000 80000 > gpurun_out/r06/size_sweep_c.txt 2>&1 || { tail gpurun_out/r06/size_sweep_c.txt; exit 1; }
cat gpurun_out/r06/size_sweep_c.txt
