"""Worker for tests/test_rccl_gpu.py: the library's RCCL transport in a world of one rank
(one GPU can host only one RCCL rank).  Runs the reference's communicator calls through the C
ABI: create_communicator -> _CAPI_get_unique_id / _CAPI_set_nccl (nccl_context.cc:13-45), the
1-float all-reduce barrier (Barrier_, :46-50), TensorP2PServer create / views / collective
destroy (tensor_p2p_cache.cc:11-118), _Test_NCCLTensorAllGather (:52-112), then a sampler and a
feature server built under the communicator."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out_path):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import dgs
    from DistGNN.dist import create_communicator
    create_communicator(1)
    res = {"world": dgs.ops._Test_GetWorldSize(), "rank": dgs.ops._Test_GetLocalRank()}
    from dgs._lib import lib
    res["barrier_rc"] = int(lib.dgs_barrier())
    indptr = torch.tensor([0, 4, 5, 5, 5, 5, 10, 10, 10, 10, 10, 10])
    sub = dgs.ops._Test_ExtractIndptr(torch.tensor([0, 3]).cuda(), indptr.cuda())
    srv = dgs.classes.TensorP2PServer(sub)
    res["p2p_view"] = srv._CAPI_get_device_tensor(0).tolist()
    res["p2p_local"] = srv._CAPI_get_local_device_tensor().tolist()
    del srv
    res["allgather"] = [t.tolist() for t in
                        dgs.ops._Test_NCCLTensorAllGather(torch.arange(5).float().cuda())]
    feat = torch.arange(100).float().reshape(10, 10)
    fs = dgs.classes.P2PCacheFeatureServer(feat, torch.tensor([0, 3]).cuda(), 0)
    res["feature_kat"] = fs._CAPI_get_feature(torch.tensor([0, 3, 5, 7]).cuda()).tolist()
    indices = torch.arange(1, 11)
    s = dgs.classes.P2PCacheSampler(indptr, indices, torch.Tensor(), torch.tensor([0, 5]), 0)
    dgs.ops._CAPI_set_random_seed(99)
    out = s._CAPI_sample_node_classifiction(torch.tensor([0, 3, 5]).cuda(), [2, 2], False)
    res["sample"] = [[f.tolist(), r.tolist(), c.tolist()] for (_, f, r, c) in out]
    del fs, s
    res["barrier_rc_end"] = int(lib.dgs_barrier())
    torch.cuda.synchronize()
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
