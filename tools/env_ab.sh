#!/bin/bash
# Same-box A/B of environment settings on the synchronous call (tools/sync_call_phases.py) and,
# unless BENCH=0, the pipelined bench (1000 steps), interleaved rounds.  Settings are
# "NAME:ENV=... ENV=..." strings ("base:" for none).
# Usage: tools/env_ab.sh OUTDIR ROUNDS "v1" "v2" ...
out=$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs DGS_CALL_TRACE=1 timeout -k 10 240 python -u tools/sync_call_phases.py \
      --calls 300 > "$out/sync_$name.$r.txt" 2>&1 \
      || { echo "sync $name $r failed"; tail -20 "$out/sync_$name.$r.txt"; exit 1; }
    bl=""
    if [ "${BENCH:-1}" != 0 ]; then
      env $envs timeout -k 10 300 python -u bench.py --steps 1000 --warmup 30 \
        --secondary none --no-cpu-baseline > "$out/bench_$name.$r.json" 2> "$out/bench_$name.$r.err" \
        || { echo "bench $name $r failed"; tail -20 "$out/bench_$name.$r.err"; exit 1; }
      bl="$out/bench_$name.$r.json"
    fi
    python - "$out/sync_$name.$r.txt" "$name" $bl <<'PY'
import json, sys
span = [l.split()[-1] for l in open(sys.argv[1]) if "GPU span" in l]
wall = [l.split()[-1] for l in open(sys.argv[1]) if "public entry point wall" in l]
s = f"[{sys.argv[2]}] sync call wall {wall[0] if wall else '?'} us, GPU span {span[0] if span else '?'} us"
if len(sys.argv) > 3:
    d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
    s += (f"; bench {d['value']/1e9:.4f} G edges/s {d['ms_per_step']*1e3:.1f} us/step, "
          f"sequential {d.get('sequential_value', 0)/1e9:.3f} G")
print(s)
PY
  done
done
