# A/B of the loader host path: ab/head is a git worktree of the previous commit built in place
# (git worktree add -f ab/head HEAD; make -C ab/head/dist-gnn_amd/csrc); run with gpurun.
set -e
mkdir -p gpurun_out/loader_ab
for r in 1 2 3 4 5; do
 for v in head new; do
  if [ $v = head ]; then d=ab/head; else d=.; fi
  timeout -k 10 120 python $d/tools/loader_host.py --scale 17 --ef 9 --fan-out 10,10 --dim 128 --steps 4000 2>&1 | grep B= >> gpurun_out/loader_ab/arxiv_$v.log
  timeout -k 10 120 python $d/tools/loader_host.py --steps 2000 2>&1 | grep B= >> gpurun_out/loader_ab/products_$v.log
 done
done
