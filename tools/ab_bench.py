"""Same-box A/B of library builds: alternates `bench.py` runs over the given libdgs_amd.so
files (DGS_AMD_LIB) and prints the median ms/step and sample span of each.  Box-to-box noise
is about 3 %, so kernel changes worth 1-2 % are only visible side by side.

    python tools/ab_bench.py --rounds 3 -- scratch/ab/libA.so scratch/ab/libB.so [-- bench args]
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    rounds = 3
    if argv[:1] == ["--rounds"]:
        rounds, argv = int(argv[1]), argv[2:]
    if argv[:1] == ["--"]:
        argv = argv[1:]
    if "--" in argv:
        i = argv.index("--")
        libs, extra = argv[:i], argv[i + 1:]
    else:
        libs, extra = argv, []
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, DGS_AMD_LIB=os.path.abspath(lib))
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"] + extra
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                sys.stderr.write(out.stderr[-2000:])
                sys.exit(out.returncode)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
            d = json.loads(line)
            iso = d.get("roofline_isolated", {}).get("frac", 0.0)
            res[lib].append((d["ms_per_step"], d["sample_span_ms_per_call"],
                             d["roofline"]["frac"], iso, d["value"]))
            print(f"round {r} {lib}: {d['ms_per_step'] * 1e3:.1f} us/step "
                  f"sample span {d['sample_span_ms_per_call'] * 1e3:.1f} us "
                  f"gather frac {d['roofline']['frac']:.3f} (isolated {iso:.3f})", flush=True)
    for lib, v in res.items():
        med = [statistics.median(x[i] for x in v) for i in range(5)]
        print(f"MEDIAN {lib}: {med[4] / 1e6:.0f} M edges/s, {med[0] * 1e3:.1f} us/step, "
              f"sample span {med[1] * 1e3:.1f} us, gather frac {med[2]:.3f}, "
              f"isolated {med[3]:.3f}")


if __name__ == "__main__":
    main()
