#!/bin/bash
# Round 4: N = 2 shared-GPU bench runs with the round-2/3 loader ordering ("old": outputs from
# the caller's stream pool) and the current one ("new"), interleaved, 300 timed steps each.
# A run that fails with an ordinary error (exit 1: e.g. the relabel range check) does not stop
# the next; a fault, abort or time limit ends the script.
set -uo pipefail
O=gpurun_out/${1:-r04n2}
RUNS=${RUNS:-3}
mkdir -p $O
rm -rf $O/oldpy && cp -r dist-gnn_amd/python $O/oldpy
python tools/r04_old_loader.py $O/oldpy/DistGNN/dataloading/prefetch.py
run() {
  local name=$1; shift
  echo "== $(date +%T) $name"
  env "$@" DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 300 \
    --warmup 5 --no-cpu-baseline --no-replicated-pass > $O/$name.log 2>&1
  local rc=$?
  grep -h "outside\|Error\|error\|^{" $O/$name.log | cut -c1-300
  echo "rc=$rc"
  case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
for i in $(seq 1 $RUNS); do
  run old_$i DGS_BENCH_PYDIR=$PWD/$O/oldpy DGS_AMD_LIB=$PWD/dist-gnn_amd/lib/libdgs_amd.so
  run new_$i X=1
done
echo "== end"
