#!/bin/bash
# Same-box A/B only (configs[1] uniform unless extra bench args after --): AB_LIBS="variants".
set -uo pipefail
O=gpurun_out/${1:-r03ab}
shift || true
mkdir -p $O
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $AB_LIBS -- "$@" > $O/ab.txt 2>&1 \
  || { tail -20 $O/ab.txt; exit 1; }
grep MEDIAN $O/ab.txt
