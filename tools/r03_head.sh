#!/bin/bash
# Head check on one MI355X: the whole GPU suite, smoke, the default bench line, the biased line,
# the N = 2 flow on one GPU, and a rocprofv3 kernel-trace of the default bench.  Every GPU step has
# its own time limit; the first failure ends the script.
set -uo pipefail
O=gpurun_out/${1:-r03h}
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step smoke
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
step bench
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
step bench-bias
timeout -k 10 400 python bench.py --bias --no-cpu-baseline > $O/bench_bias.log 2>&1 \
  || { tail -20 $O/bench_bias.log; exit 1; }
step n2
DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 100 --warmup 5 \
  --no-cpu-baseline > $O/n2.log 2>&1 || { tail -20 $O/n2.log; exit 1; }
step rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 bench.py --no-cpu-baseline > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
step done
step rocprof-bias
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_bias -- \
  python3 bench.py --no-cpu-baseline --bias > $O/stats_bias.log 2>&1 || { tail -20 $O/stats_bias.log; exit 1; }
step done-bias
if [ -n "${AB_LIBS:-}" ]; then
  step ab-uniform
  timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $AB_LIBS > $O/ab_uniform.txt 2>&1 \
    || { tail -20 $O/ab_uniform.txt; exit 1; }
  grep MEDIAN $O/ab_uniform.txt
fi
step end
