#!/bin/bash
# Round 4 GPU call runner: bash tools/r04_run.sh NAME step [step ...]
# Steps: pytest (all GPU tests) | pytest:<file or node> | smoke | probe (N = 2 old/new loader) |
#        n2 (N = 2 shared-device bench, default layout) | n4 | bench (N = 1 default line) |
#        bias (N = 1 biased line) | papers | papersbias | rocprof (kernel stats of the N = 1 bench)
# A step that fails with an ordinary error (rc 1) does not stop the next; a fault, abort or time
# limit ends the call.
set -uo pipefail
N=$1; shift
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
for step in "$@"; do
  echo "== $(date +%T) $step"
  case $step in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; ok $rc ;;
    pytest:*)
      f=${step#pytest:}; tag=$(echo $f | tr '/:[]' '____')
      timeout -k 10 600 python -u -m pytest $f -m gpu -x -v --timeout 300 \
        --timeout-method thread > $O/pytest_$tag.log 2>&1; rc=$?; tail -4 $O/pytest_$tag.log; ok $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -2 $O/smoke.log; ok $rc ;;
    probe)
      RUNS=${RUNS:-3} bash tools/r04_n2_probe.sh $N/n2; ok $? ;;
    n2|n4)
      k=${step#n}
      DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus $k --steps 300 \
        --warmup 10 > $O/bench_$step.json 2> $O/bench_$step.err; rc=$?
      tail -3 $O/bench_$step.err; cut -c1-300 $O/bench_$step.json; ok $rc ;;
    bench)
      timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?
      cut -c1-300 $O/bench.json; ok $rc ;;
    bias)
      timeout -k 10 300 python bench.py --bias --no-cpu-baseline > $O/bench_bias.json \
        2> $O/bench_bias.err; rc=$?; cut -c1-300 $O/bench_bias.json; ok $rc ;;
    papers)
      timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --no-cpu-baseline \
        > $O/bench_papers.json 2> $O/bench_papers.err; rc=$?; cut -c1-300 $O/bench_papers.json; ok $rc ;;
    papersbias)
      timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --bias --no-cpu-baseline \
        > $O/bench_papers_bias.json 2> $O/bench_papers_bias.err; rc=$?
      cut -c1-300 $O/bench_papers_bias.json; ok $rc ;;
    rocprof)
      (cd /tmp && export TMPDIR=/tmp) ; export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py \
        --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
      cut -c1-200 $O/bench_rocprof.json; ok $rc ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "== end $(date +%T)"
