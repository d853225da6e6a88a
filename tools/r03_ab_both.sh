#!/bin/bash
# Loader/sampler parity tests with the tree's build, then same-box A/Bs of the builds given on the
# uniform and the biased products-like lines.   bash tools/r03_ab_both.sh OUT libA.so libB.so ...
set -uo pipefail
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_prefetch_gpu.py tests/test_fullsize_gpu.py tests/test_stream_wait_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- "$@" > $O/ab_uniform.txt 2>&1 || { tail -20 $O/ab_uniform.txt; exit 1; }
grep MEDIAN $O/ab_uniform.txt
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- "$@" -- --bias --steps 300 > $O/ab_bias.txt 2>&1 || { tail -20 $O/ab_bias.txt; exit 1; }
grep MEDIAN $O/ab_bias.txt
