#!/bin/bash
# VALU PMC pass of each lib/variants build (GPU box); one rocprofv3 run per variant.
set -o pipefail
for v in ${@:-w4 f32}; do
  HLC_LIB=$PWD/hashgraph-like-consensus_amd/lib/variants/libhlc_$v.so bash tools/pmc_quick.sh var_$v 2>&1 | grep k_rec_main | sed "s/^/$v /" || exit 1
done
