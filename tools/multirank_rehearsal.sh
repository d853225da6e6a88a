#!/bin/bash
# The N = 2 bench flow rehearsed on a one-GPU box: two torchrun ranks share cuda:0 (gloo process
# group, DGS_BENCH_SHARE_DEVICE=1), replicated and --shard (v mod 2 caches read through IPC):
#   gpurun -- 'bash tools/multirank_rehearsal.sh r02'
set -euo pipefail
R=${1:-r02}
O=gpurun_out/$R
mkdir -p $O
export DGS_BENCH_SHARE_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 10 > $O/bench_n2_replicated.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 200 --warmup 10 --shard > $O/bench_n2_shard.log 2>&1
