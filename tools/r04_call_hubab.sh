#!/bin/bash
# Round 4: same-box A/B of the uniform hub kernel's work split (DGS_HUB_DYN sixteenths drawn from
# per-XCD pools) and grid (DGS_HUB_BLOCKS; 1536 = 6 waves per SIMD is the default).
set -uo pipefail
L=dist-gnn_amd/lib/libdgs_amd.so
AB_ROUNDS=${AB_ROUNDS:-5} AB_VARIANTS="$L $L,DGS_HUB_DYN=4 $L,DGS_HUB_DYN=8 $L,DGS_HUB_BLOCKS=1024" \
  bash tools/r04_run.sh ${1:-r04_hubab} ab
