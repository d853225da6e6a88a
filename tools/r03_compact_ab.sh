#!/bin/bash
# Compact row-table gather: the feature-server GPU tests with the tree's build, then the N = 2
# shared-GPU flow (hot-shard: table gather) for each build given, interleaved, 3 rounds.
set -uo pipefail
O=gpurun_out/${1:-r03ct}
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "feature or shard or multirank or prefetch or gather or fullsize or server" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    DGS_AMD_LIB="$GRAFT_REPO_ROOT/$lib" DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 300 --warmup 10 --no-cpu-baseline > $O/${n}_$r.log 2>&1 || { tail -5 $O/${n}_$r.log; exit 1; }
    python3 -c "
import json;l=[x for x in open('$O/${n}_$r.log') if x.startswith('{')][-1];d=json.loads(l);print('$n round $r', round(d['value']/1e6), 'M frac', round(d['roofline']['frac'],3), 'iso', round(d['roofline_isolated']['frac'],3), 'mb', round(d['roofline_microbench']['frac'],3))"
  done
done
