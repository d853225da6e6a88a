#!/bin/bash
# Round 4: the N = 4 and N = 8 bench flows rehearsed with every rank on the one GPU (gloo setup
# collectives, one /dev/shm host graph): the round-4 self-check (setup all-gather with
# rank-dependent lengths, first batches bit-exact against the replicated services) and the
# xGMI feature-shard pass at the driver's rank counts.
set -uo pipefail
O=gpurun_out/r04_ranks
mkdir -p $O
for k in 4 8; do
  DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python bench.py --gpus $k --steps 100 --warmup 10 \
    > $O/bench_n$k.json 2> $O/bench_n$k.err; rc=$?
  grep "self-check" $O/bench_n$k.err; cut -c1-200 $O/bench_n$k.json
  [ $rc -eq 0 ] || { tail -20 $O/bench_n$k.err; exit $rc; }
done
