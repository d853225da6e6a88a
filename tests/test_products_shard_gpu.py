"""BASELINE configs[2]'s layout at the products-like size (RMAT scale 21, edge factor 59:
N = 2,097,152, E = 123,731,968, d = 100): a hot-node cache of the 20 % highest in-degree
nodes sharded over two ranks (hot[rank::2]) for the sampler's structure and the P2P feature
server, all other rows zero-copy from pinned host memory.  The two ranks share cuda:0 (peer
rows through the IPC-mapped block of the other rank; setup over gloo); each runs two batches
of 1024 seeds through PrefetchLoader.

Checked bit-exact against the oracle: every hop's frontier and relabelled COO of both ranks
(the cache placement must not change a single pick: rowwise_sampling_p2p.cu:19-92 keeps K2's
RNG coordinates), and in the workers the gathered rows (local, peer and host rows,
feature_ops.cu:38-73) and labels against the host arrays."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FAN_OUT = [15, 10, 5]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def run():
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr_d, indices_d = rmat_csc_torch(21, 59, seed=20261015, device=dev)
    n = indptr_d.numel() - 1
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats = torch.randn(n, 100, generator=gen, device=dev).cpu()
    labels = torch.randint(0, 47, (n,), generator=gen, device=dev).cpu()
    indeg = torch.bincount(indices_d, minlength=n)
    hot = torch.sort(indeg, descending=True, stable=True).indices[: (n + 4) // 5].cpu()
    indptr, indices = indptr_d.cpu(), indices_d.cpu()
    del indptr_d, indices_d, indeg
    torch.cuda.empty_cache()
    g = torch.Generator()
    g.manual_seed(2)
    train = torch.randperm(n, generator=g)[: n // 10]
    world, seed = 2, 4242
    batches = [[train[(2 * r + b) * 1024:(2 * r + b + 1) * 1024].tolist() for b in range(2)]
               for r in range(world)]
    with tempfile.TemporaryDirectory() as td:
        for name, t in (("indptr", indptr), ("indices", indices), ("feats", feats),
                        ("labels", labels), ("hot", hot)):
            t.numpy().tofile(os.path.join(td, f"{name}.bin"))
        json.dump({"n": n, "e": indices.numel(), "dim": 100, "batches": batches, "seed": seed},
                  open(os.path.join(td, "meta.json"), "w"))
        port = _free_port()
        procs = []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), LOCAL_RANK="0")
            procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "shard_worker.py"),
                                           td, td], env=env))
        rcs = [p.wait(timeout=300) for p in procs]
        assert rcs == [0] * world, rcs
        res = [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]
        arr = [dict(np.load(os.path.join(td, f"r{r}.npz"))) for r in range(world)]
    return dict(indptr=indptr.numpy(), indices=indices.numpy(), batches=batches, seed=seed,
                res=res, arr=arr, world=world)


def test_sharded_hot_cache_blocks_match_oracle(run):
    ip, ix = run["indptr"], run["indices"]
    for r in range(run["world"]):
        ls = O.launch_seeds(run["seed"] + r, 3 * 2)
        for b, seeds in enumerate(run["batches"][r]):
            exp = O.node_classification_sample(np.array(seeds, dtype=np.int64), ip, ix, FAN_OUT,
                                               False, ls[3 * b:3 * b + 3])
            for h, (_, ef, er, ec) in enumerate(exp):
                a = run["arr"][r]
                assert np.array_equal(a[f"b{b}_h{h}_f"], ef), (r, b, h)
                assert np.array_equal(a[f"b{b}_h{h}_r"], er), (r, b, h)
                assert np.array_equal(a[f"b{b}_h{h}_c"], ec), (r, b, h)


def test_sharded_hot_cache_gather_exact(run):
    for res in run["res"]:
        assert res["gather_ok"] == [True, True] and res["labels_ok"] == [True, True]
        assert res["layout"] == -1  # a partial cache: per-node address table
        # host rows were part of it (the sampled frontier reaches beyond the hot 20 %)
        assert 0 < res["host_rows"] < res["rows"]
