#!/bin/bash
# Round-6 A/B call: (1) the host-buffer entry with far-node inputs under each staging placement
# (tools/numa_ab.py); (2) the 128-B R-table arm against the shipped build, headline
# leg, 3 alternating rounds (tools/ab_arms.sh); (3) both arms' k_rec_main counters (tools/ab_pmc.sh).
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u tools/numa_ab.py --steps 10 --rounds 3 > gpurun_out/r06/numa_ab.txt 2> gpurun_out/r06/numa_ab.err || { tail gpurun_out/r06/numa_ab.err; exit 1; }
bash tools/ab_arms.sh tab128 > gpurun_out/r06/ab_tab128_headline.txt 2>&1 || { tail gpurun_out/r06/ab_tab128_headline.txt; exit 1; }
bash tools/ab_pmc.sh tab128 > gpurun_out/r06/ab_tab128_pmc.txt 2>&1 || { tail gpurun_out/r06/ab_tab128_pmc.txt; exit 1; }
cat gpurun_out/r06/ab_tab128_headline.txt gpurun_out/r06/ab_tab128_pmc.txt
tail -2 gpurun_out/r06/numa_ab.txt
