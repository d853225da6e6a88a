#!/bin/bash
# Round 4 call k3: the final head check first (every GPU test, smoke, the default bench line with
# the CPU baseline, its rocprofv3 kernel stats, the biased lines, the N = 2 shared-device
# self-check), then the uniform hub kernel's balance: parity of ab/pad (hub rows register padding
# units, DGS_HUB_PAD, that the static split counts and the kernel skips) and a same-box A/B:
# ab/pre (bd82fbd), HEAD 1536 / 1024 / 3072 workgroups, ab/pad with 1 and 2 padding units.
set -uo pipefail
O=gpurun_out/r04_k3
mkdir -p $O
L=dist-gnn_amd/lib/libdgs_amd.so
bash tools/r04_run.sh r04_final pytest smoke bench rocprof bias papersbias n2 || exit $?
DGS_AMD_LIB=$PWD/ab/pad/libdgs_amd.so DGS_HUB_PAD=2 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_parity.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_pad2.log 2>&1; prc=$?; tail -2 $O/pytest_pad2.log
case $prc in 0|1) ;; *) exit $prc ;; esac
P=ab/pad/libdgs_amd.so
V="ab/pre/libdgs_amd.so $L $L,DGS_HUB_BLOCKS=1024 $L,DGS_HUB_BLOCKS=3072"
[ $prc -eq 0 ] && V="$V $P,DGS_HUB_PAD=1 $P,DGS_HUB_PAD=2"
AB_ROUNDS=3 AB_VARIANTS="$V" bash tools/r04_run.sh r04_k3_hubgrid ab
