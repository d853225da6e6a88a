"""World-size-2 gloo tests on CPU for the distributed host logic: communicator bootstrap
(DistGNN.dist.create_communicator), the bench's seed partition and its max/sum-over-ranks
reduction.  The RCCL join itself needs GPUs; it is recorded here through a stub."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)


def _communicator_worker(rank, world, port, q):
    _init(rank, world, port)
    import dgs
    from DistGNN.dist import create_communicator
    calls = []
    dgs.ops._CAPI_get_unique_id = lambda: [11 * (i + 1) for i in range(16)]
    dgs.ops._CAPI_set_nccl = lambda n, ids, r: calls.append((n, list(ids), r))
    create_communicator(world)
    q.put((rank, calls))
    dist.destroy_process_group()


def _bench_worker(rank, world, port, q):
    _init(rank, world, port)
    import bench
    train = torch.arange(101)
    part = bench.seed_slice(train, rank, world)
    out = bench.reduce_over_ranks(dist, torch.device("cpu"), 1.0 + rank, 10 * (rank + 1),
                                  3 + rank, 808 * (3 + rank))
    q.put((rank, part.tolist(), out))
    dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


def test_create_communicator_world2():
    res = _run(_communicator_worker)
    ids = [11 * (i + 1) for i in range(16)]
    assert res == [(0, [(2, ids, 0)]), (1, [(2, ids, 1)])]


def test_bench_partition_and_reduction_world2():
    res = _run(_bench_worker)
    parts = [r[1] for r in res]
    assert parts[0] == list(range(0, 51)) and parts[1] == list(range(51, 101))
    for _, _, (elapsed, edges, rows, gbytes) in res:
        assert elapsed == 2.0 and edges == 30.0 and rows == 7.0 and gbytes == 808 * 7
