#!/bin/bash
# The driver's short bench (20 timed steps after 5 warm-up steps) repeated under variants given
# as environment settings ("-" = none), interleaved: value, host step gaps and the allocator's
# hipMalloc calls inside the timed region.  Run on the GPU box:
#   bash tools/short_run.sh ROUNDS "-" "DGS_EXACT_ALLOC=1"
set -euo pipefail
R=$1; shift
O=gpurun_out/short
mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    if [ "$v" = "-" ]; then e=(); else e=($v); fi
    env "${e[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/v${i}_$r.log 2>&1
    python - "$O/v${i}_$r.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
g = d["host_step_gap_ms"]
print(f"{sys.argv[2]:24s} {d['value'] / 1e9:.3f} G  mallocs {d.get('allocator_mallocs_in_timed_region')}"
      f"  gaps p50 {g['p50']:.3f} p90 {g['p90']:.3f} max {g['max']:.3f}", flush=True)
PY
  done
done
