#!/bin/bash
# One GPU call: the named test files first (each step under its own time limit), then the whole
# GPU suite and smoke(); stops at the first failure.  Usage: tools/gpu_suite.sh OUTDIR [files...]
out=$1; shift
mkdir -p "$out"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread \
    > "$out/focused.log" 2>&1 || { echo "focused tests failed"; tail -40 "$out/focused.log"; exit 1; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.log" 2>&1 || { echo "gpu suite failed"; tail -60 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
