#!/bin/bash
# Round 4: same-box A/B of the biased hub merge's batches per memory round trip
# (ab/ilp1 = one batch per round trip, the round-3 form; HEAD = 4).
set -uo pipefail
L=dist-gnn_amd/lib/libdgs_amd.so
AB_ROUNDS=${AB_ROUNDS:-3} AB_VARIANTS="ab/ilp1/libdgs_amd.so $L" AB_ARGS="--bias" \
  bash tools/r04_run.sh r04_mergeab ab || exit $?
AB_ROUNDS=${AB_ROUNDS:-3} AB_VARIANTS="ab/ilp1/libdgs_amd.so $L" AB_ARGS="--bias --scale 27 --ef 12 --dim 128" \
  AB_TIMEOUT=600 bash tools/r04_run.sh r04_mergeab_papers ab
