"""Worker for tests/test_multirank_gpu.py: one rank of a 2-rank job whose ranks share cuda:0.

Setup collectives run over gloo (dgs.ops._CAPI_set_host_comm); the caches are sharded (node v
on rank v % 2), so every rank reads half of its rows through the peer's IPC-mapped block.
Results are written as JSON for the parent test to compare with the oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out_path):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import dgs
    dgs.ops._CAPI_set_host_comm()
    res = {"rank": rank, "world": dgs.ops._Test_GetWorldSize(),
           "local_rank": dgs.ops._Test_GetLocalRank()}

    # reference tests/test_p2p_server.py + test_feature_server.py known answers
    indptr = torch.tensor([0, 4, 5, 5, 5, 5, 10, 10, 10, 10, 10, 10])
    cache = torch.tensor([0, 3]) if rank == 0 else torch.tensor([3, 5])
    sub = dgs.ops._Test_ExtractIndptr(cache.cuda(), indptr.cuda())
    srv = dgs.classes.TensorP2PServer(sub)
    res["p2p_views"] = [srv._CAPI_get_device_tensor(i).tolist() for i in range(world)]
    feat = torch.arange(0, 100, 1).float().reshape(10, 10)
    fs = dgs.classes.P2PCacheFeatureServer(feat, cache.cuda(), 0)
    res["feature_kat"] = fs._CAPI_get_feature(torch.tensor([0, 3, 5, 7]).cuda()).tolist()
    gathered = dgs.ops._Test_NCCLTensorAllGather(torch.full((rank + 2,), float(rank)).cuda())
    res["allgather"] = [g.tolist() for g in gathered]

    # sharded sampler / feature server on a random graph with hubs
    rng = np.random.default_rng(0)
    n = 600
    degs = rng.integers(0, 70, n)
    degs[:4] = [0, 3000, 1500, 20]
    ip = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    ix = rng.integers(0, n, int(ip[-1])).astype(np.int64)
    probs = (rng.random(ix.size) + 0.05).astype(np.float32)
    mine = np.arange(rank, n, world)
    for bias in (False, True):
        s = dgs.classes.P2PCacheSampler(torch.from_numpy(ip), torch.from_numpy(ix),
                                        torch.from_numpy(probs) if bias else torch.Tensor(),
                                        torch.from_numpy(mine), 0)
        seeds = rng.permutation(n)[:80]
        dgs.ops._CAPI_set_random_seed(777)
        out = s._CAPI_sample_node_classifiction(torch.from_numpy(seeds).cuda(), [10, 5], False)
        res[f"sample_bias{int(bias)}"] = {
            "seeds": seeds.tolist(),
            "hops": [[f.tolist(), r.tolist(), c.tolist()] for (_, f, r, c) in out]}
        key, idx, devid = s._local_cache_map_compact()
        res[f"map_bias{int(bias)}"] = [key.tolist(), idx.tolist(), devid.tolist()]
        key, idx, devid = s._CAPI_get_local_cache_hashmap_tensors()
        res[f"refmap_bias{int(bias)}"] = [key.tolist(), idx.tolist(), devid.tolist()]
        del s
    data = rng.standard_normal((n, 33)).astype(np.float32)
    fs2 = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(data), torch.from_numpy(mine), 0)
    q = rng.integers(0, n, 500)
    got = fs2._CAPI_get_feature(torch.from_numpy(q).cuda()).cpu().numpy()
    res["gather_ok"] = bool(np.array_equal(got, data[q]))
    res["gather_layout"] = fs2._layout()
    torch.cuda.synchronize()
    del fs, fs2, srv
    dist.barrier()
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
