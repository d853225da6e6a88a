"""Worker for tests/test_multirank_gpu.py's setup-failure tests: one rank of a 2-rank job sharing
cuda:0.  Mode "export": rank 1 reports a failed IPC export (DGS_TEST_IPC_EXPORT_FAIL=1).  Mode
"args": rank 1 passes an out-of-range cache id to each service.  Mode "build": rank 1's service
builds fail (DGS_TEST_BUILD_FAIL=1).  Every rank must raise from the service constructor naming
rank 1 -- none may wait in a setup collective -- and the process
group must still work afterwards."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out_path, mode):
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    import dgs
    dgs.ops._CAPI_set_host_comm()
    msgs = []
    feat = torch.arange(40, dtype=torch.float32).reshape(10, 4)
    bad = torch.tensor([1, 2]) if rank == 0 else torch.tensor([1, 99])
    ip = torch.arange(0, 21, 2)
    ix = torch.arange(20) % 10
    if mode == "build":
        calls = [lambda: dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.tensor([1]), 0),
                 lambda: dgs.classes.P2PCacheFeatureServer(feat, torch.tensor([1, 2]), 0)]
    elif mode == "export":
        calls = [lambda: dgs.classes.TensorP2PServer(torch.arange(100, device="cuda")),
                 lambda: dgs.classes.P2PCacheFeatureServer(feat, torch.tensor([1, 2]), 0)]
    else:
        calls = [lambda: dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), bad, 0),
                 lambda: dgs.classes.P2PCacheFeatureServer(feat, bad, 0)]
    for call in calls:
        try:
            call()
            msgs.append("no error")
        except RuntimeError as e:
            msgs.append(str(e).replace("\n", " "))
    if mode != "export":  # the library and the process group are usable afterwards
        srv = dgs.classes.TensorP2PServer(torch.arange(10, device="cuda") + 100 * rank)
        peer = srv._CAPI_get_device_tensor(1 - rank).cpu().tolist()
        msgs.append("after: ok" if peer == [100 * (1 - rank) + i for i in range(10)]
                    else f"after: wrong peer view {peer}")
        del srv
    msg = "\n".join(msgs)
    dist.barrier()  # both ranks got here: nobody is left waiting in the exchange
    with open(out_path, "w") as f:
        f.write(msg)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
