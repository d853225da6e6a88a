#!/bin/bash
# configs[3] shape (papers100M-like, degree-weighted biased, d = 128): the pipelined bench line
# and a rocprofv3 kernel trace of the sequential loop.
set -uo pipefail
O=gpurun_out/${1:-r03pp}
mkdir -p $O
echo "== $(date +%T) bench"
timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --bias --steps 300 --no-cpu-baseline \
  > $O/bench_papers_bias.log 2>&1 || { tail -20 $O/bench_papers_bias.log; exit 1; }
grep '^{' $O/bench_papers_bias.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== $(date +%T) rocprof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_papers_bias -- \
  python3 bench.py --scale 27 --ef 12 --dim 128 --bias --depth 1 --steps 100 --warmup 10 \
  --seq-calls 10 --no-cpu-baseline > $O/stats_papers_bias.log 2>&1 || { tail -20 $O/stats_papers_bias.log; exit 1; }
python3 tools/prof_summary.py $(ls $O/stats_papers_bias/*/*kernel_stats.csv) 14
echo "== $(date +%T) end"
