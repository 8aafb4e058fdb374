#!/bin/bash
# Round-6 A/B: the table rescale's entry and z-ratio loads issued at the top of each step
# (HLC_BUILD_PREFETCH=1, lib/variants/libhlc_bpf.so) against the shipped build, headline leg, 3 rounds.
set -o pipefail
mkdir -p gpurun_out/r06
bash tools/ab_arms.sh bpf > gpurun_out/r06/ab_bpf_headline.txt 2>&1 || { tail gpurun_out/r06/ab_bpf_headline.txt; exit 1; }
cat gpurun_out/r06/ab_bpf_headline.txt
