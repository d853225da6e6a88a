#!/bin/bash
# Same-box A/B of host-side (Python) changes on the host-bound arxiv-like line: the tree's packages
# against the copy in $PYDIR_B, interleaved, R rounds.   bash tools/r03_py_ab.sh OUT PYDIR_B [R]
set -uo pipefail
O=gpurun_out/$1
B=$2
R=${3:-4}
mkdir -p $O
export DGS_AMD_LIB="$GRAFT_REPO_ROOT/dist-gnn_amd/lib/libdgs_amd.so"
for r in $(seq 1 $R); do
  for v in tree alt; do
    if [ $v = alt ]; then export DGS_BENCH_PYDIR="$GRAFT_REPO_ROOT/$B"; else unset DGS_BENCH_PYDIR; fi
    timeout -k 10 200 python bench.py --scale 17 --ef 9 --dim 128 --fan-out 10,10 --no-cpu-baseline \
      > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    echo "$v $r: $(grep -o '"value": [0-9.]*' $O/${v}_$r.log | head -1)"
  done
done
