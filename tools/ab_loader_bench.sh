#!/bin/bash
# Same-box A/B of the loader host path (round 2, profiles/r02_ab_loader_*.txt): ab/head is a git
# worktree of the commit to compare against, built in place
#   git worktree add -f ab/head <commit>; make -C ab/head/dist-gnn_amd/csrc
# then on the GPU box: bash tools/ab_loader_bench.sh OUT_DIR ROUNDS.  Each round runs, for head
# and for this tree: bench.py 20 steps (the driver's short run), bench.py 200 steps, and
# tools/loader_host.py on the arxiv-like config.
set -euo pipefail
O=${1:-gpurun_out/ab_loader}; R=${2:-5}
mkdir -p $O
val() { grep '^{' | python -c "import json,sys; print(round(json.loads(sys.stdin.read())['value']/1e9,3))"; }
for r in $(seq 1 $R); do for v in head new; do
  if [ $v = head ]; then d=ab/head; else d=.; fi
  echo "$v short $( (cd $d && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline) 2>/dev/null | val)" >> $O/res.txt
  echo "$v long $( (cd $d && timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline) 2>/dev/null | val)" >> $O/res.txt
  timeout -k 10 120 python $d/tools/loader_host.py --scale 17 --ef 9 --fan-out 10,10 --dim 128 --steps 4000 2>&1 | grep B= | sed "s/^/$v arxiv /" >> $O/res.txt
done; done
