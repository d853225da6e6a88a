"""Worker for tests/test_multirank_gpu.py::test_failed_export_raises_on_every_rank: one rank of a
2-rank job sharing cuda:0 whose rank 1 reports a failed IPC export (DGS_TEST_IPC_EXPORT_FAIL=1).
Every rank must raise from the service constructor naming rank 1 -- none may wait in the
exchange -- and the process group must still work afterwards."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out_path):
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    import dgs
    dgs.ops._CAPI_set_host_comm()
    msg = "no error"
    try:
        dgs.classes.TensorP2PServer(torch.arange(100, device="cuda"))
    except RuntimeError as e:
        msg = str(e)
    feat = torch.arange(40, dtype=torch.float32).reshape(10, 4)
    try:
        dgs.classes.P2PCacheFeatureServer(feat, torch.tensor([1, 2]), 0)
    except RuntimeError as e:
        msg += "\n" + str(e)
    dist.barrier()  # both ranks got here: nobody is left waiting in the exchange
    with open(out_path, "w") as f:
        f.write(msg)


if __name__ == "__main__":
    main(sys.argv[1])
