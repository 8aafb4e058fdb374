#!/bin/bash
# A/B build of the recovery AND prehash objects with extra defines:
#   bash tools/build_variant2.sh NAME "-DFOO -DBAR"  ->  lib/variants/libhlc_NAME.so
set -e
cd "$(dirname "$0")/../hashgraph-like-consensus_amd"
NAME=$1; DEFS=$2
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable"
mkdir -p build/variants lib/variants
/opt/rocm/bin/hipcc $F $DEFS -c csrc/hlc_recover.hip -o build/variants/rec_$NAME.o &
/opt/rocm/bin/hipcc $F $DEFS -c csrc/hlc_prehash.hip -o build/variants/pre_$NAME.o &
wait
/opt/rocm/bin/hipcc $F -shared -o lib/variants/libhlc_$NAME.so build/hlc_api.o build/hlc_wire.o build/hlc_stream.o build/hlc_synth.o build/variants/rec_$NAME.o build/variants/pre_$NAME.o
