#!/bin/bash
# Round 4 head check 3 (after the stream-kernel changes) + uniform hub-reservoir grid A/B
# (1536 = 6 waves per SIMD, the default, against 1024 / 768 workgroups) + hub-kernel workgroup
# stamps inside the pipeline (DGS_PROF_HUB: late starts / uneven finishes of the fixed shares).
set -uo pipefail
bash tools/r04_run.sh r04_head3 pytest smoke bench n2 bias papersbias || exit $?
O=gpurun_out/r04_head3
for v in "" "--bias"; do
  DGS_PROF_HUB=1 DGS_PROF_DETAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline $v \
    > $O/hubstamps$v.json 2> $O/hubstamps$v.err || exit $?
  grep "dgs prof" $O/hubstamps$v.err | tail -4
done
# the hub kernel's dynamic pools (DGS_HUB_DYN sixteenths; default 0 = fixed shares): parity
DGS_HUB_DYN=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_hubdyn8.log 2>&1 || exit $?
tail -2 $O/pytest_hubdyn8.log
for v in 4 8; do
  DGS_HUB_DYN=$v DGS_PROF_HUB=1 DGS_PROF_DETAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline \
    > $O/hubstamps_dyn$v.json 2> $O/hubstamps_dyn$v.err || exit $?
  grep "dgs prof" $O/hubstamps_dyn$v.err | tail -3; cut -c1-200 $O/hubstamps_dyn$v.json
done
