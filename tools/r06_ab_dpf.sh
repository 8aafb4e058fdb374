#!/bin/bash
# Round-6 A/B: the u2 R chain's digit words loaded at the window top and read after its doublings
# (HLC_DIGIT_PREFETCH=1, lib/variants/libhlc_dpf.so) against the shipped build, headline leg, 3 rounds.
set -o pipefail
mkdir -p gpurun_out/r06
bash tools/ab_arms.sh dpf > gpurun_out/r06/ab_dpf_headline.txt 2>&1 || { tail gpurun_out/r06/ab_dpf_headline.txt; exit 1; }
cat gpurun_out/r06/ab_dpf_headline.txt
