"""How many 32-edge groups of biased hub rows could skip their probability loads with a
per-group maximum weight (VERDICT r05 "Next round" 3), simulated on the CPU.

k_bias_stream's half-wave covers one aligned 32-edge group per step; a group's probability load
can be skipped only when every lane's draw is rejected by the linear bound evaluated with the
group's maximum weight p_max (sound: the bound's threshold falls as p grows, since T <= 0).  For
hub rows (degree > 1024) of a degree-weighted RMAT graph this draws the reference-distributed
u per edge, takes T as the k-th largest key of a 4096-edge sample (as k_bias_boot), and counts
groups with at least one surviving lane under exact p and under p_max."""
import argparse
import sys

import numpy as np

sys.path.insert(0, "dist-gnn_amd/python")
from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_numpy  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=20)
ap.add_argument("--ef", type=int, default=12)
ap.add_argument("--k", type=int, default=15)
ap.add_argument("--rows", type=int, default=300)
a = ap.parse_args()
ip, ix = rmat_csc_numpy(a.scale, a.ef, seed=5)
probs = degree_probs(ip, ix)
deg = np.diff(ip)
hubs = np.nonzero(deg > 1024)[0]
rng = np.random.default_rng(1)
groups = surv_p = surv_pmax = edges = passed = 0
for r in rng.choice(hubs, min(a.rows, hubs.size), replace=False):
    p = probs[ip[r]:ip[r + 1]].astype(np.float64)
    d = p.size
    u = rng.random(d)
    keys = np.log2(u) / p
    samp = keys[rng.choice(d, 4096, replace=False)] if d > 4096 else keys
    cx = np.sort(samp)[-a.k] * np.log(2)
    pass_e = u >= 1 + p * cx  # the stream kernel's linear bound (its float margins aside)
    ng, pad = (d + 31) // 32, (-d) % 32
    pm = np.concatenate([p, np.zeros(pad)]).reshape(ng, 32).max(1)
    uu = np.concatenate([u, -np.ones(pad)]).reshape(ng, 32)
    surv_pmax += int(np.any(uu >= (1 + pm * cx)[:, None], axis=1).sum())
    surv_p += int(np.any(np.concatenate([pass_e, np.zeros(pad, bool)]).reshape(ng, 32), 1).sum())
    groups, edges, passed = groups + ng, edges + d, passed + int(pass_e.sum())
print(f"RMAT scale {a.scale} ef {a.ef}, degree-weighted, k = {a.k}: {hubs.size} hub rows, "
      f"{min(a.rows, hubs.size)} simulated, {groups} groups of 32 edges")
print(f"edges passing the linear bound: {passed / edges:.4f}")
print(f"groups with a surviving lane: exact p {surv_p / groups:.3f}, p_max bound "
      f"{surv_pmax / groups:.3f} -> loads skippable with p_max: {1 - surv_pmax / groups:.3f}")
