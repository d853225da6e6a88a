#!/bin/bash
# Round 4 call k3: all GPU tests at HEAD (lane moves, sorted first groups, merge ILP, stamps),
# then a same-box A/B of the uniform hub kernel grid: ab/pre (bd82fbd), HEAD 1536 / 1280 / 1024.
set -uo pipefail
O=gpurun_out/r04_k3
mkdir -p $O
L=dist-gnn_amd/lib/libdgs_amd.so
bash tools/r04_run.sh r04_k3 pytest || exit $?
AB_ROUNDS=5 AB_VARIANTS="ab/pre/libdgs_amd.so $L $L,DGS_HUB_BLOCKS=1280 $L,DGS_HUB_BLOCKS=1024" \
  bash tools/r04_run.sh r04_k3_hubgrid ab
