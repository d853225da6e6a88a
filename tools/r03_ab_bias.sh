#!/bin/bash
# Biased path A/B on the GPU box: the biased GPU tests with this build, then a same-box A/B
# (products-like, degree-weighted, B = 1024, 300 steps) of the library builds given, and a
# per-kernel rocprofv3 comparison of the first and last build (sequential loop).
#   bash tools/r03_ab_bias.sh OUT libA.so libB.so ... [-- extra bench args]
set -uo pipefail
O=gpurun_out/$1
shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p $O
echo "== $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "bias or papers" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== $(date +%T) A/B"
timeout -k 10 1200 python tools/ab_bench.py --rounds 3 -- "${libs[@]}" -- --bias --steps 300 "$@" \
  > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep MEDIAN $O/ab.txt
echo "== $(date +%T) kernels"
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
first="${libs[0]}"; last="${libs[${#libs[@]}-1]}"
files=()
for lib in "$first" "$last"; do
  n=$(echo "$lib" | tr '/,=' '___')
  (
    IFS=, read -ra parts <<< "$lib"
    export DGS_AMD_LIB="$R/${parts[0]}"
    for kv in "${parts[@]:1}"; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/k_$n -- python3 bench.py --no-cpu-baseline --bias --depth 1 --steps 200 --warmup 10 "$@" \
      > $O/k_$n.log 2>&1
  ) || { tail -20 $O/k_$n.log; exit 1; }
  files+=("$(find $O/k_$n -name "*kernel_stats.csv" | head -1)")
done
python3 tools/prof_summary.py --compare "${files[@]}" > $O/kernels.txt; head -14 $O/kernels.txt
