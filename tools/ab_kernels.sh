#!/bin/bash
# Same-box per-kernel A/B: rocprofv3 kernel-trace stats of bench.py under each library build
# (DGS_AMD_LIB), then one table of average kernel durations.  Run on the GPU box:
#   bash tools/ab_kernels.sh scratch/ab/libA.so scratch/ab/libB.so [-- bench args]
set -euo pipefail
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
O=gpurun_out/abk
rm -rf $O && mkdir -p $O
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
i=0
files=()
for lib in "${libs[@]}"; do
  n=$i.$(basename "$lib" .so)
  i=$((i + 1))
  DGS_AMD_LIB="$R/$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/$n -- python3 bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1
  files+=("$(find $O/$n -name "*kernel_stats.csv" | head -1)")
done
echo "columns: ${libs[*]}"
python3 tools/prof_summary.py --compare "${files[@]}"
