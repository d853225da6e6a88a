#!/bin/bash
# Loader host-cost check: the prefetch GPU tests, then the host-bound arxiv-like line twice and the
# products-like uniform line once.
set -uo pipefail
O=gpurun_out/${1:-r03lc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_prefetch_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --scale 17 --ef 9 --dim 128 --fan-out 10,10 --no-cpu-baseline > $O/arxiv_$r.log 2>&1 || { tail -5 $O/arxiv_$r.log; exit 1; }
  echo "arxiv $r: $(grep -o '"value": [0-9.]*' $O/arxiv_$r.log | head -1)"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/products.log 2>&1 || { tail -5 $O/products.log; exit 1; }
echo "products: $(grep -o '"value": [0-9.]*' $O/products.log | head -1)"
