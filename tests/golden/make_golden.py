"""Regenerates the committed fixtures under tests/golden/.

  rng_kat.json        Philox4x32-10 streams from torch's header-only at::philox_engine and
                      std::mt19937_64 / uniform_int_distribution outputs from libstdc++
                      (gen_rng_kat.cpp, compiled with g++ here) -- independent anchors for
                      the oracle's curand / launch-seed restatement.
  reference_kats.json Known answers hand-derived from the reference's own test scripts
                      (tests/test_extract.py, test_p2p_server.py, test_feature_server.py,
                      test_sampler_{uniform,bias}.py of CommediaJW/Dist-GNN): inputs + expected.
  sampler_golden.npz  Small seeded graphs and the oracle's outputs for every sampler variant,
                      relabel and the multi-hop sample (regression pin of the oracle itself).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

from oracle import oracle as O  # noqa: E402


def rng_kat():
    import torch
    inc = os.path.join(os.path.dirname(torch.__file__), "include")
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "gen_rng_kat")
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", inc,
                               os.path.join(HERE, "gen_rng_kat.cpp"), "-o", exe])
        out = subprocess.check_output([exe]).decode()
    data = json.loads(out)
    # Random123 published known answers for philox4x32_10 (kat_vectors)
    data["random123_philox4x32_10"] = [
        {"ctr": [0, 0, 0, 0], "key": [0, 0],
         "out": [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]},
        {"ctr": [0xffffffff] * 4, "key": [0xffffffff] * 2,
         "out": [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]},
        {"ctr": [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
         "key": [0xa4093822, 0x299f31d0],
         "out": [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]},
    ]
    data["mt19937_64_10000th_default_seed"] = "9981545732273789042"
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(data, f, indent=1)


def reference_kats():
    indptr = [0, 4, 5, 5, 5, 5, 10, 10, 10, 10, 10, 10]
    indices = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
    probs = [0.1, 0.2, 0.3, 0.4, 0.5, 0.1, 0.2, 0.3, 0.4, 0.5]
    kats = {
        "toy_graph": {"indptr": indptr, "indices": indices, "probs": probs},
        # tests/test_extract.py: cache [0, 1, 5]
        "extract": {"cache_nids": [0, 1, 5], "sub_indptr": [0, 4, 5, 10],
                    "sub_indices": [1, 2, 3, 4, 5, 6, 7, 8, 9, 10],
                    "sub_probs": [0.1, 0.2, 0.3, 0.4, 0.5, 0.1, 0.2, 0.3, 0.4, 0.5]},
        # tests/test_p2p_server.py: rank0 caches [0, 3], rank1 caches [3, 5]
        "p2p_server": {"rank_cache_nids": [[0, 3], [3, 5]],
                       "rank_sub_indptr": [[0, 4, 4], [0, 0, 5]]},
        # tests/test_feature_server.py: features arange(100).reshape(10, 10)
        "feature_server": {"rank_cache_nids": [[0, 3], [3, 5]], "query": [0, 3, 5, 7],
                           "expected": [list(range(0, 10)), list(range(30, 40)),
                                        list(range(50, 60)), list(range(70, 80))]},
        # tests/test_sampler_{uniform,bias}.py: seeds [0, 3, 5], fan-out [2, 2]
        "sampler": {"seeds": [0, 3, 5], "fan_out": [2, 2],
                    "neighbours": {"0": [1, 2, 3, 4], "3": [], "5": [6, 7, 8, 9, 10]},
                    "frontier_prefix": [0, 3, 5]},
    }
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)


def sampler_golden():
    from DistGNN.dataloading.synthetic import rmat_csc_numpy, degree_probs
    out = {}
    indptr, indices = rmat_csc_numpy(10, 8, seed=20261015)
    probs = np.abs(np.random.default_rng(7).standard_normal(indices.size)).astype(np.float32)
    dprobs = degree_probs(indptr, indices)
    seeds = np.random.default_rng(2).permutation(indptr.size - 1)[:300].astype(np.int64)
    out["indptr"], out["indices"], out["probs"], out["dprobs"], out["seeds"] = \
        indptr, indices, probs, dprobs, seeds
    ls = O.launch_seeds(7, 16)
    out["launch_seeds"] = np.array(ls, dtype=np.uint64)
    i = 0
    for k in (3, 5, 15, 40):
        for rep in (0, 1):
            r, c = O.sample_uniform(seeds, indptr, indices, k, rep, ls[i % 16])
            out[f"uniform_k{k}_r{rep}_row"], out[f"uniform_k{k}_r{rep}_col"] = r, c
            r, c = O.sample_bias(seeds, indptr, indices, probs, k, rep, ls[i % 16])
            out[f"bias_k{k}_r{rep}_row"], out[f"bias_k{k}_r{rep}_col"] = r, c
            i += 1
    res = O.node_classification_sample(seeds[:64], indptr, indices, [15, 10, 5], False, ls[:3])
    for h, (s, f, r, c) in enumerate(res):
        out[f"nc_h{h}_seeds"], out[f"nc_h{h}_frontier"] = s, f
        out[f"nc_h{h}_row"], out[f"nc_h{h}_col"] = r, c
    np.savez_compressed(os.path.join(HERE, "sampler_golden.npz"), **out)


if __name__ == "__main__":
    O.build()
    rng_kat()
    reference_kats()
    sampler_golden()
    print("fixtures written to", HERE)
