#!/bin/bash
# Round 4 call k3: the final head check first (every GPU test, smoke, the default bench line with
# the CPU baseline, its rocprofv3 kernel stats, the biased lines, the N = 2 shared-device
# self-check), then a same-box A/B of the uniform hub kernel grid: ab/pre (bd82fbd), HEAD
# 1536 / 1024 / 3072 / 6144 workgroups (more, smaller workgroups: the dispatcher balances late
# starts).
set -uo pipefail
L=dist-gnn_amd/lib/libdgs_amd.so
bash tools/r04_run.sh r04_final pytest smoke bench rocprof bias papersbias n2 || exit $?
AB_ROUNDS=3 AB_VARIANTS="ab/pre/libdgs_amd.so $L $L,DGS_HUB_BLOCKS=1024 $L,DGS_HUB_BLOCKS=3072 $L,DGS_HUB_BLOCKS=6144" \
  bash tools/r04_run.sh r04_k3_hubgrid ab
