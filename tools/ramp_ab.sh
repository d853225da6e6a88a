#!/bin/bash
# Same-box A/B of the driver's 20-step bench (python bench.py --steps 20 --warmup 5) over
# settings given as "NAME:ENV=... ENV=..." strings (STEPS=n for other step counts), interleaved rounds; prints value, step-gap
# max and the loader trace of the first steps.  Usage: tools/ramp_ab.sh OUTDIR ROUNDS "v1" "v2" ..
out=$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs DGS_PREFETCH_TRACE=1 timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 5 \
      --secondary none --no-cpu-baseline --seq-calls 5 > "$out/$name.$r.json" 2> "$out/$name.$r.err" \
      || { echo "run $name $r failed"; tail -20 "$out/$name.$r.err"; exit 1; }
    python - "$out/$name.$r.json" "$out/$name.$r.err" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tr = [l for l in open(sys.argv[2]) if "loader trace" in l]
res = [int(x.split('@')[1]) for x in tr[0].split(':', 1)[1].split() if x.startswith('result@')] if tr else []
print(f"[{sys.argv[3]}] {d['value']/1e9:.3f} G {d['ms_per_step']*1e3:.1f} us/step gap max "
      f"{d['host_step_gap_ms']['max']:.3f}  results@ " + " ".join(map(str, res)))
PY
  done
done
