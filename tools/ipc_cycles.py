"""IPC export / import cycles of TensorP2PServer between torchrun ranks sharing cuda:0 (round-6
probe of an intermittent hipIpcGetMemHandle 'invalid argument' after ~16k multi-rank service
builds): blocks of random small and large sizes, created and destroyed in a loop; the first
failure prints its cycle and size.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29535 tools/ipc_cycles.py [--seconds 150] [--max-bytes 65536]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--max-bytes", type=int, default=65536)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    import dgs
    dgs.ops._CAPI_set_host_comm()
    rng = np.random.default_rng(7)  # the same sizes on every rank
    t0 = time.time()
    i = 0
    hist = {}
    while True:
        stop = torch.tensor([time.time() - t0 > a.seconds], dtype=torch.int32)
        dist.all_reduce(stop, op=dist.ReduceOp.MAX)
        if stop.item():
            break
        nb = int(rng.integers(1, a.max_bytes + 1))
        t = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        try:
            s = dgs.classes.TensorP2PServer(t)
            del s
        except Exception as e:  # noqa: BLE001
            print(f"[ipc] rank {rank}: failed at cycle {i}, block of {nb} B: {e}", flush=True)
            os._exit(3)
        hist[nb.bit_length()] = hist.get(nb.bit_length(), 0) + 1
        i += 1
        if i % 5000 == 0 and rank == 0:
            print(f"[ipc] {i} cycles {time.time() - t0:.0f} s", flush=True)
    print(f"[ipc] rank {rank}: {i} cycles ok; blocks by bit length {sorted(hist.items())}",
          flush=True)


if __name__ == "__main__":
    main()
