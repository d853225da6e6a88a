"""Same-box A/B of library builds and runtime settings: alternates `bench.py` runs over the
given variants and prints the median ms/step, sample span and gather roofline of each.  Box-to-box
noise is about 3 %, so kernel changes worth 1-2 % are only visible side by side.

A variant is a libdgs_amd.so path (DGS_AMD_LIB), optionally followed by comma-separated
environment settings: `ab/u8/libdgs_amd.so,DGS_HUB_BLOCKS=1024`; a setting that starts with
`--` is a bench argument instead (`ab/u8/libdgs_amd.so,--depth=4,GPU_MAX_HW_QUEUES=8`).

    python tools/ab_bench.py --rounds 3 -- ab/a/libdgs_amd.so ab/b/libdgs_amd.so [-- bench args]
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def variant_env(spec):
    parts = spec.split(",")
    env = dict(os.environ, DGS_AMD_LIB=os.path.abspath(parts[0]))
    for kv in parts[1:]:
        if kv.startswith("--"):
            continue
        k, v = kv.split("=", 1)
        env[k] = v
    return env


def variant_args(spec):
    return [kv for kv in spec.split(",")[1:] if kv.startswith("--")]


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
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"] + extra + variant_args(lib)
            if "--secondary" not in extra:
                cmd += ["--secondary", "none"]
            out = subprocess.run(cmd, env=variant_env(lib), capture_output=True, text=True,
                                 timeout=int(os.environ.get("AB_TIMEOUT", "300")))
            if out.returncode != 0:
                sys.stderr.write(out.stderr[-2000:])
                sys.exit(out.returncode)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
            d = json.loads(line)
            iso = d.get("roofline_isolated", {}).get("frac", 0.0)
            res[lib].append((d["ms_per_step"], d["sample_span_ms_per_call"],
                             d["roofline"]["frac"], iso, d["value"],
                             d.get("sequential_value", 0.0)))
            print(f"round {r} {lib}: {d['ms_per_step'] * 1e3:.1f} us/step "
                  f"sample span {d['sample_span_ms_per_call'] * 1e3:.1f} us "
                  f"gather frac {d['roofline']['frac']:.3f} (isolated {iso:.3f}) "
                  f"sequential {d.get('sequential_value', 0.0) / 1e6:.0f} M", flush=True)
    for lib, v in res.items():
        med = [statistics.median(x[i] for x in v) for i in range(6)]
        print(f"MEDIAN {lib}: {med[4] / 1e6:.0f} M edges/s, {med[0] * 1e3:.1f} us/step, "
              f"sample span {med[1] * 1e3:.1f} us, gather frac {med[2]:.3f}, "
              f"isolated {med[3]:.3f}, sequential {med[5] / 1e6:.0f} M edges/s")


if __name__ == "__main__":
    main()
