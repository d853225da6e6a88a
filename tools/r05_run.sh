#!/bin/bash
# Round 5 GPU call runner: bash tools/r05_run.sh NAME step [step ...]
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
    n2|n4|n8)
      k=${step#n}
      DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus $k --steps 300 \
        --warmup 10 > $O/bench_$step.json 2> $O/bench_$step.err; rc=$?
      tail -3 $O/bench_$step.err; cut -c1-300 $O/bench_$step.json; ok $rc ;;
    bench)
      timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?
      cut -c1-300 $O/bench.json; ok $rc ;;
    bias)
      timeout -k 10 300 python bench.py --bias --no-cpu-baseline > $O/bench_bias.json \
        2> $O/bench_bias.err; rc=$?; cut -c1-300 $O/bench_bias.json; ok $rc ;;
    papers)
      timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --no-cpu-baseline \
        > $O/bench_papers.json 2> $O/bench_papers.err; rc=$?; cut -c1-300 $O/bench_papers.json; ok $rc ;;
    papersbias)
      timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --bias --no-cpu-baseline \
        ${PB_ARGS:-} > $O/bench_papers_bias.json 2> $O/bench_papers_bias.err; rc=$?
      cut -c1-300 $O/bench_papers_bias.json; tail -8 $O/bench_papers_bias.err; ok $rc ;;
    driverbench)
      # the driver's own command, timed
      t0=$(date +%s.%N)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 \
        > $O/driver_bench.json 2> $O/driver_bench.err; rc=$?
      echo "driver bench wall: $(python3 -c "import time; print(round(time.time() - $t0, 1))") s" | tee $O/driver_bench_wall.txt
      cut -c1-300 $O/driver_bench.json; tail -12 $O/driver_bench.err; ok $rc ;;
    rocprof)
      (cd /tmp && export TMPDIR=/tmp) ; export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py \
        --no-cpu-baseline --secondary none ${PROF_ARGS:-} > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
      cut -c1-200 $O/bench_rocprof.json; ok $rc ;;
    detail)
      # workgroup stamps of the gather and hub kernels inside the pipeline (DGS_PROF_DETAIL)
      DGS_PROF_DETAIL=1 DGS_PROF_HUB=1 timeout -k 10 600 python bench.py --no-cpu-baseline \
        --secondary none ${DETAIL_ARGS:-} > $O/detail.json 2> $O/detail.err; rc=$?
      grep "dgs prof" $O/detail.err | tail -12; ok $rc ;;
    ab)
      # same-box A/B: AB_VARIANTS (space-separated ab_bench variants), AB_ARGS (bench args)
      timeout -k 10 1000 python tools/ab_bench.py --rounds ${AB_ROUNDS:-3} -- $AB_VARIANTS \
        -- ${AB_ARGS:-} > $O/ab.txt 2>&1; rc=$?; grep MEDIAN $O/ab.txt; ok $rc ;;
    synchost)
      timeout -k 10 300 python tools/r04_sync_host.py > $O/sync_host.txt 2>&1; rc=$?
      cat $O/sync_host.txt | tail -12; ok $rc ;;
    pmcpipe)
      # SQ counters per kernel, pipelined (depth 3) and sequential (depth 1) uniform loops
      export TMPDIR=/tmp
      for d in 3 1; do
        timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
          SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU \
          --output-format csv -d $O/pmc_d$d -- python3 bench.py --depth $d --steps 200 \
          --warmup 10 --seq-calls 3 --no-cpu-baseline > $O/pmc_d$d.log 2>&1; rc=$?
        ok $rc
        python3 tools/pmc_kernels.py "$(find $O/pmc_d$d -name '*counter_collection.csv' | head -n 1)" \
          > $O/pmc_d${d}_summary.txt; head -12 $O/pmc_d${d}_summary.txt | cut -c1-250
      done ;;
    calltrace)
      # kernel trace of the sequential loop: one sample call's kernels in stream order
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/calls -- \
        python3 bench.py --depth 1 --steps 100 --warmup 10 --seq-calls 3 --no-cpu-baseline \
        ${CALL_ARGS:-} > $O/calls.log 2>&1; rc=$?; ok $rc
      python3 tools/call_breakdown.py "$(ls -t $(find $O/calls -name '*kernel_trace.csv') | head -n 1)" \
        > $O/call_breakdown.txt; cat $O/call_breakdown.txt | tail -25 ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "== end $(date +%T)"
