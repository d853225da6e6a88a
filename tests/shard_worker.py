"""Worker for tests/test_products_shard_gpu.py: one rank of BASELINE configs[2]'s layout at the
products-like size, with the ranks sharing cuda:0 (setup collectives over gloo through
dgs.ops._CAPI_set_host_comm; RCCL refuses two ranks on one device).

The HBM caches hold the 20 % highest in-degree nodes, sharded v mod W by position in that list
(hot[rank::W], for the sampler's structure and the feature server alike); every other node's
neighbour ids and feature row are read zero-copy from the pinned host arrays.  Each rank runs
its own seed batches through PrefetchLoader (3 in flight) and writes the blocks for the parent
to check against the oracle; gathered rows and labels are checked here against the host
arrays (byte-exact), host rows included."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FAN_OUT = [15, 10, 5]


def main(indir, out_dir):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import dgs
    from DistGNN.dataloading import PrefetchLoader
    dgs.ops._CAPI_set_host_comm()
    meta = json.load(open(os.path.join(indir, "meta.json")))

    def load(name, dtype, shape):
        return torch.from_numpy(np.fromfile(os.path.join(indir, name), dtype=dtype)
                                .reshape(shape))

    n, e, d = meta["n"], meta["e"], meta["dim"]
    indptr = load("indptr.bin", np.int64, (n + 1,))
    indices = load("indices.bin", np.int64, (e,))
    feats = load("feats.bin", np.float32, (n, d))
    labels = load("labels.bin", np.int64, (n,))
    hot = load("hot.bin", np.int64, (-1,))
    mine = hot[rank::world].contiguous()
    sampler = dgs.classes.P2PCacheSampler(indptr, indices, torch.Tensor(), mine, 0)
    server = dgs.classes.P2PCacheFeatureServer(feats, mine, 0)
    batches = [torch.from_numpy(np.array(b, dtype=np.int64)).cuda()
               for b in meta["batches"][rank]]
    dgs.ops._CAPI_set_random_seed(meta["seed"] + rank)
    labels_d = labels.cuda()
    res = {"rank": rank, "layout": server._layout(), "gather_ok": [], "labels_ok": [],
           "host_rows": 0, "rows": 0}
    cached = torch.zeros(n, dtype=torch.bool)
    cached[hot] = True
    arrays = {}
    for b, (blocks, x, y) in enumerate(PrefetchLoader(sampler, batches, FAN_OUT, server=server,
                                                      labels=labels_d, depth=3)):
        front = blocks[-1][1].cpu()
        res["gather_ok"].append(bool(torch.equal(x.cpu().view(torch.int32),
                                                 feats[front].view(torch.int32))))
        res["labels_ok"].append(bool(torch.equal(y.cpu(), labels[batches[b].cpu()])))
        res["host_rows"] += int((~cached[front]).sum())
        res["rows"] += int(front.numel())
        for h, (s, f, r, c) in enumerate(blocks):
            arrays[f"b{b}_h{h}_f"] = f.cpu().numpy()
            arrays[f"b{b}_h{h}_r"] = r.cpu().numpy()
            arrays[f"b{b}_h{h}_c"] = c.cpu().numpy()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **arrays)
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    del sampler, server  # collective destructors
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
