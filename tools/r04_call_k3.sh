#!/bin/bash
# Round 4 call k3: all GPU tests at HEAD (lane moves, sorted first groups, merge ILP, stamps),
# then a same-box A/B of the uniform hub kernel grid: ab/pre (bd82fbd), HEAD 1536 / 1024 / 3072 / 6144 (more, smaller workgroups: the dispatcher balances late starts).
set -uo pipefail
O=gpurun_out/r04_k3
mkdir -p $O
L=dist-gnn_amd/lib/libdgs_amd.so
bash tools/r04_run.sh r04_k3 pytest || exit $?
AB_ROUNDS=4 AB_VARIANTS="ab/pre/libdgs_amd.so $L $L,DGS_HUB_BLOCKS=1024 $L,DGS_HUB_BLOCKS=3072 $L,DGS_HUB_BLOCKS=6144" \
  bash tools/r04_run.sh r04_k3_hubgrid ab
