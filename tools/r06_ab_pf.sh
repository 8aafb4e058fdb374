#!/bin/bash
# Round-6 A/B: the latency-bound stages' loads issued ahead of their use.  pld: k_rec_prep's forward pass in
# three round trips per vote (HLC_PREP_LOADS=1); pld2: also its backward reload in two (=2); fin: k_rec_final's
# state and Z loads for a lane's 8 votes at once, the Zs kept for the backward pass (HLC_FIN_LOADS=1); pf: pld2 +
# fin.  Headline leg, 3 alternating rounds; then the config-4 shard leg for default / pf (occupancy check).
set -o pipefail
mkdir -p gpurun_out/r06
bash tools/ab_arms.sh pld pld2 fin pf > gpurun_out/r06/ab_pf_headline.txt 2>&1 || { tail gpurun_out/r06/ab_pf_headline.txt; exit 1; }
cat gpurun_out/r06/ab_pf_headline.txt
AB_MODE=c4 bash tools/ab_arms.sh pf > gpurun_out/r06/ab_pf_c4.txt 2>&1 || { tail gpurun_out/r06/ab_pf_c4.txt; exit 1; }
cat gpurun_out/r06/ab_pf_c4.txt
