#!/bin/bash
# round 5: the driver's 20-step run -- pipeline fill diagnostics (loader trace) under variants
O=gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  for V in "" "DGS_PREFETCH_RAMP_SYNC=1" "DGS_BENCH_GC_EARLY=1" "DGS_PREFETCH_RAMP_SYNC=1 DGS_BENCH_GC_EARLY=1"; do
    env $V DGS_PREFETCH_TRACE=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 \
      --secondary none --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 - "$V" $O/b.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().splitlines()[-1])
print(f"[{sys.argv[1] or 'default'}] {d['value'] / 1e9:.3f} G mallocs {d['allocator_mallocs_in_timed_region']} "
      f"gap p50 {d['host_step_gap_ms']['p50']:.3f} max {d['host_step_gap_ms']['max']:.3f}")
PY
    grep "loader trace" $O/b.err | cut -c1-220
  done
done
