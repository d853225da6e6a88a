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


def self_exchange(out_path):
    """DGS_COMM_SELF_EXCHANGE=1: the own rank is a peer of the all-gathers, so a world of one
    runs ncclAllGather of the sizes and the grouped ncclSend / ncclRecv payload exchange
    (nccl_context.cc:52-112) on this GPU.  Rank-dependent payloads; the received bytes are
    checked against what was sent."""
    os.environ["DGS_COMM_SELF_EXCHANGE"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import ctypes
    import dgs
    from dgs._lib import c_i64, check, i64_array, lib, stream_ptr, vp_array
    from DistGNN.dist import create_communicator
    create_communicator(1)
    rank = dgs.ops._Test_GetLocalRank()
    res = {"world": dgs.ops._Test_GetWorldSize()}
    sizes = (c_i64 * 1)()
    check(lib.dgs_allgather_sizes(12345 + rank, sizes))
    res["sizes"] = [int(sizes[0])]
    # a 3 MB + 5 B payload into a separate receive buffer
    g = torch.Generator(device="cuda")
    g.manual_seed(17 + rank)
    n = 3 * (1 << 20) + 5
    send = torch.randint(0, 256, (n,), generator=g, device="cuda", dtype=torch.uint8)
    recv = torch.zeros(n, dtype=torch.uint8, device="cuda")
    check(lib.dgs_allgather_bytes(ctypes.c_void_p(send.data_ptr()), n,
                                  vp_array([recv.data_ptr()]), i64_array([n]), stream_ptr()))
    torch.cuda.synchronize()
    res["bytes_equal"] = bool(torch.equal(recv, send))
    res["bytes_nonzero"] = int((recv != 0).sum())
    # the reference's _Test_NCCLTensorAllGather (receive buffer aliases the payload)
    t = torch.arange(7, dtype=torch.float32, device="cuda") + 100 * rank + 0.5
    res["allgather"] = [x.tolist() for x in dgs.ops._Test_NCCLTensorAllGather(t)]
    # services built with the exchange on (their cache lists travel through it)
    feat = torch.arange(100).float().reshape(10, 10)
    fs = dgs.classes.P2PCacheFeatureServer(feat, torch.tensor([0, 3]).cuda(), 0)
    res["feature_kat"] = fs._CAPI_get_feature(torch.tensor([0, 3, 5, 7]).cuda()).tolist()
    del fs
    res["barrier_rc"] = int(lib.dgs_barrier())
    torch.cuda.synchronize()
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


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
    if len(sys.argv) > 2 and sys.argv[2] == "self":
        self_exchange(sys.argv[1])
    else:
        main(sys.argv[1])
