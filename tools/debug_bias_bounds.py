"""Prints the inputs where the biased filters' bounds fail (debug companion of
tests/test_gpu_parity.py::test_bias_filter_bounds_are_sound; same inputs)."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "dist-gnn_amd", "python"))
import numpy as np, torch
import dgs
from oracle import oracle as O
import importlib.util
spec = importlib.util.spec_from_file_location("t", "tests/test_gpu_parity.py")
rng = np.random.default_rng(31)
n = 1 << 22
x = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
ex = np.array([0, 1, 2, 255, 256, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 1, 2 ** 32 - 2, 2 ** 32 - 128,
               2 ** 32 - 129, 2 ** 32 - 256, 2 ** 32 - 512, 2 ** 32 - 4608, 2 ** 32 - 4609,
               2 ** 32 - 8192], dtype=np.uint64)
p = np.exp(rng.uniform(np.log(1e-6), np.log(1e6), n)).astype(np.float32)
p[1::3] = rng.integers(1, 200000, p[1::3].size).astype(np.float32)
ep = np.array([0.0, -0.0, -1.0, 1e-45, 1e-40, 7.8e-31, 7.888609052210118e-31, 1e-30, 0.5, 1.0,
               1e30, 1.2676506002282294e30, 1.3e30, 1e38, np.inf, np.nan], dtype=np.float32)
gx, gp = np.meshgrid(ex, ep)
m = gx.size
x[:m], p[:m] = gx.ravel(), gp.ravel()
x[m:2 * m], p[m:2 * m] = gx.ravel(), rng.uniform(0.5, 3.0, m).astype(np.float32)
u = O.curand_uniform_of(x)
key = O.ares_keys(u, p)
fac = np.array([1.0, 1.0 + 2 ** -24, 1.0 - 2 ** -24, 1.0 + 2 ** -20, 1.0 - 2 ** -20,
                1.0 + 2 ** -16, 1.0 - 2 ** -16, 1.0 + 2 ** -12, 1.0 - 2 ** -12, 1.5, 0.5, 4.0],
               dtype=np.float32)
thr = key * fac[rng.integers(0, fac.size, n)]
ties = rng.random(n) < 0.2
thr[ties] = key[ties]
bad = ~np.isfinite(thr)
thr[bad] = -np.exp(rng.uniform(np.log(1e-9), np.log(1e3), int(bad.sum()))).astype(np.float32)
thr[:16] = 0.0
cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
gk, gl, gf = dgs.ops._Test_BiasKeyBounds(cu(x.astype(np.int64)), cu(p), cu(thr))
gk, gl, gf = gk.cpu().numpy(), gl.cpu().numpy(), gf.cpu().numpy()
print("key mismatch", int((gk.view(np.uint32) != key.view(np.uint32)).sum()))
print("klow > key", int((gl > gk).sum()))
for bit in (1, 2):
    fired = (gf & bit) != 0
    wrong = fired & ~(gk < thr)
    print("bit", bit, "fired", fired.mean(), "wrong", int(wrong.sum()))
    idx = np.nonzero(wrong)[0][:25]
    for i in idx:
        print(f"  i={i} x={int(x[i])} u={u[i]!r} p={p[i]!r} key={gk[i]!r} thr={thr[i]!r} klow={gl[i]!r}")
