#!/bin/bash
# Round-3 check on the GPU box: GPU tests (default build), the biased tests again with the
# wave-worker biased hub kernel, the N = 2 bench flow on one GPU, the default bench line, and a
# same-box A/B of the biased hub kernels.  Every step has its own time limit; the first failure
# ends the script.
set -uo pipefail
O=gpurun_out/${1:-r03c}
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step pytest-bias-wave
DGS_BIAS_HUB_WAVE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 \
  --timeout-method thread -k "bias or papers" > $O/pytest_wave.log 2>&1 \
  || { tail -30 $O/pytest_wave.log; exit 1; }
tail -2 $O/pytest_wave.log
step n2
DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 \
  > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
step bench
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
step ab-bias
L=dist-gnn_amd/lib/libdgs_amd.so
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- ab/base/libdgs_amd.so $L $L,DGS_BIAS_HUB_WAVE=1 -- --bias \
  --steps 300 > $O/ab_bias.txt 2>&1 || { tail -20 $O/ab_bias.txt; exit 1; }
tail -3 $O/ab_bias.txt
step done
