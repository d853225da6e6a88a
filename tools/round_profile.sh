#!/bin/bash
# Round-end measurement on one MI355X (run from the repo root on the GPU box, e.g.
# gpurun -- 'bash tools/round_profile.sh r01').  Every GPU step has its own time limit and the
# steps are chained with set -e.  Outputs land in gpurun_out/; the summaries worth keeping are
# copied into profiles/ by tools/collect_profiles.sh.
set -euo pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
# PART=runs: the GPU suite, smoke and the bench lines; PART=prof: the rocprofv3 passes (each part
# fits one gpurun call); default both
PART=${2:-all}
if [ "$PART" != prof ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
timeout -k 10 400 python bench.py --bias > $O/bench_bias.log 2>&1
timeout -k 10 400 python bench.py --batch 8192 --no-cpu-baseline > $O/bench_b8192.log 2>&1
timeout -k 10 400 python bench.py --batch 8192 --bias --no-cpu-baseline > $O/bench_b8192_bias.log 2>&1
fi
[ "$PART" = runs ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 bench.py --no-cpu-baseline --secondary none > $O/stats.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench_fetch -- python3 bench.py --no-cpu-baseline --secondary none --steps 10 --warmup 2 > $O/pmc_bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_bench_write -- python3 bench.py --no-cpu-baseline --secondary none --steps 10 --warmup 2 > $O/pmc_bench_write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_fetch -- python3 tools/gather_calib.py > $O/pmc_calib_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_write -- python3 tools/gather_calib.py > $O/pmc_calib_write.log 2>&1
python tools/pmc_traffic.py $O $O/gather_pmc.json > $O/pmc_traffic.log 2>&1
