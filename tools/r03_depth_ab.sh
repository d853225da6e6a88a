#!/bin/bash
# Biased pipeline depth / hardware-queue A/B on one box: 3 interleaved rounds of
#   depth 3 | depth 4 | depth 4 with GPU_MAX_HW_QUEUES=8   (products-like, degree-weighted, B=1024)
set -uo pipefail
O=gpurun_out/${1:-r03dq}
mkdir -p $O
B="bench.py --bias --no-cpu-baseline --steps 300 --warmup 20"
for r in 1 2 3; do
  for v in d3 d4 d4q8; do
    case $v in
      d3) timeout -k 10 240 python $B --depth 3 > $O/${v}_$r.log 2>&1 ;;
      d4) timeout -k 10 240 python $B --depth 4 > $O/${v}_$r.log 2>&1 ;;
      d4q8) GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python $B --depth 4 > $O/${v}_$r.log 2>&1 ;;
    esac
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/${v}_$r.log; exit $rc; }
    echo "$v round $r: $(grep -o '"value": [0-9.]*' $O/${v}_$r.log | head -1)"
  done
done
