#!/bin/bash
# Copies the summaries of a round's GPU runs (tools/round_profile.sh + tools/configs_run.sh,
# merged back into gpurun_out/$R) into profiles/ under the round's prefix.
set -euo pipefail
R=${1:-r01}
O=gpurun_out/$R
P=profiles
line() { grep -h '^{' "$1" | tail -n 1; }
line $O/bench.log > $P/${R}_bench_line.json
line $O/bench_bias.log > $P/${R}_bench_bias_line.json
line $O/bench_b8192.log > $P/${R}_bench_b8192_line.json
line $O/bench_b8192_bias.log > $P/${R}_bench_b8192_bias_line.json
[ -f $O/bench_arxiv.log ] && line $O/bench_arxiv.log > $P/${R}_bench_arxiv_line.json
[ -f $O/bench_rmat1b.log ] && line $O/bench_rmat1b.log > $P/${R}_bench_rmat1b_line.json
line $O/stats.log > $P/${R}_bench_under_rocprof_line.json
# newest files: gpurun_out/ keeps the traces of earlier runs of the same round
newest() { ls -t $(find "$1" -name "$2") | head -n 1; }
S=$(newest $O/stats '*kernel_stats.csv')
T=$(newest $O/stats '*kernel_trace.csv')
cp "$S" $P/${R}_bench_kernel_stats.csv
python tools/prof_summary.py "$S" 40 > $P/${R}_bench_kernel_stats_summary.txt
python tools/timeline.py "$T" --warmup 30 --steps 1000 > $P/${R}_timeline_uniform.txt
if [ -d $O/stats_bias ]; then
  python tools/timeline.py "$(newest $O/stats_bias '*kernel_trace.csv')" \
    > $P/${R}_timeline_bias_sequential.txt
fi
cp $O/gather_pmc.json $P/${R}_gather_pmc.json
cp $O/gather_pmc.json $P/gather_pmc.json
tail -n 1 $O/pytest_gpu.log > $P/${R}_pytest_gpu_summary.txt
cat $O/smoke.log | grep -v amdgpu.ids >> $P/${R}_pytest_gpu_summary.txt
