"""Host logic of bench.py (no GPU): rank-count checks, workload placement per mode, and the
one-host-copy input sharing of N > 1 runs (gloo world 2 on CPU)."""
import glob
import os
import socket
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_world_mismatch_fails_loudly():
    args = bench.parse(["--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.check_world(args, "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=1 but --gpus 4"):
        bench.check_world(args, None)
    assert bench.check_world(bench.parse(["--gpus", "2"]), "2") == 2
    assert bench.check_world(bench.parse([]), None) == 1


def test_spawn_refuses_more_ranks_than_gpus(monkeypatch):
    monkeypatch.delenv("DGS_BENCH_SHARE_DEVICE", raising=False)
    with pytest.raises(SystemExit, match="GPUs are visible"):
        bench.launch_ranks(max(torch.cuda.device_count(), 1) + 1, [])


def test_modes_and_cache_lists():
    assert bench.resolve_mode(bench.parse([]), 1) == "replicated"
    assert bench.resolve_mode(bench.parse(["--gpus", "8"]), 8) == "hot-shard"
    assert bench.parse(["--shard"]).mode == "shard"
    N, W = 37, 4
    allv = torch.arange(N)
    for r in range(W):
        s, f = bench.cache_lists("replicated", N, r, W, None)
        assert torch.equal(s, allv) and torch.equal(f, allv)
        s, f = bench.cache_lists("feature-shard", N, r, W, None)
        assert torch.equal(s, allv) and torch.equal(f, torch.arange(r, N, W))
        s, f = bench.cache_lists("shard", N, r, W, None)
        assert torch.equal(s, torch.arange(r, N, W)) and torch.equal(f, s)
    hot = torch.tensor([5, 1, 9, 3, 7])
    s, f = bench.cache_lists("feature-shard", N, 1, 2, hot)
    assert torch.equal(s, hot) and torch.equal(f, torch.tensor([1, 3]))
    # the union of the sharded feature lists is every node exactly once
    parts = torch.cat([bench.cache_lists("feature-shard", N, r, W, None)[1] for r in range(W)])
    assert torch.equal(torch.sort(parts).values, allv)
    # hot-shard: the hot nodes on every GPU, every other node on exactly one
    hot_feat = torch.tensor([4, 17, 30])
    seen = torch.zeros(N, dtype=torch.int64)
    for r in range(W):
        s, f = bench.cache_lists("hot-shard", N, r, W, None, hot_feat)
        assert torch.equal(s, allv) and torch.equal(f[:3], hot_feat)
        assert torch.unique(f).numel() == f.numel()
        seen[f] += 1
    assert torch.equal(seen[hot_feat], torch.full((3,), W))
    cold = torch.ones(N, dtype=torch.bool)
    cold[hot_feat] = False
    assert torch.equal(seen[cold], torch.ones(int(cold.sum()), dtype=torch.int64))


def test_workload_names():
    assert bench.workload_name(21, 59) == "products-like"
    assert bench.workload_name(27, 12) == "papers100M-like"
    assert bench.workload_name(26, 16) == "RMAT-1B"
    assert bench.workload_name(17, 9) == "arxiv-like"
    assert bench.workload_name(12, 3) == "RMAT scale 12 ef 3"


def test_baseline_threads_rule(monkeypatch):
    monkeypatch.delenv("DGS_CPU_THREADS", raising=False)
    info = {"cgroup_cpu_quota": None, "usable_cpus": 256}
    assert bench.baseline_threads(info) == (32, "usable CPUs / 8 GPUs per node")
    info["cgroup_cpu_quota"] = 16.0
    assert bench.baseline_threads(info)[0] == 16
    monkeypatch.setenv("DGS_CPU_THREADS", "3")
    assert bench.baseline_threads(info) == (3, "DGS_CPU_THREADS")


def _shared_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = bench.parse(["--gpus", str(world), "--scale", "8", "--ef", "4", "--dim", "6",
                        "--bias"])
    inp, how = bench.shared_inputs(args, torch.device("cpu"), dist, rank, f"test{port}")
    torch.save({k: (v.clone() if v is not None else None) for k, v in inp.items()} | {"how": how},
               f"{out}/r{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


def test_shared_inputs_one_host_copy(tmp_path):
    """Local rank 0 builds the inputs once; both ranks map the same /dev/shm pages and see
    identical tensors; the file names are gone once every rank has mapped them."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_shared_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["how"].startswith("one copy per node")
    for k in ("indptr", "indices", "probs", "feats", "labels"):
        assert torch.equal(r0[k], r1[k]), k
    n = 1 << 8
    assert r0["indptr"].numel() == n + 1 and r0["indices"].numel() == n * 4
    assert r0["feats"].shape == (n, 6)
    deg = torch.bincount(r0["indices"], minlength=n)
    assert torch.equal(r0["probs"], (1 + deg[r0["indices"]]).float())
    assert not glob.glob(f"/dev/shm/dgs_bench_test{port}_*")


def _selfcheck_worker(rank, world, port, corrupt, out):
    """bench.multi_rank_self_check's all-gather leg and cross-rank verdict, with the library's
    all-gather stood in by a gloo one (optionally corrupting one payload on rank 1)."""
    import types

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(t):
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([t.numel()]))
        m = max(int(x) for x in sizes)
        pad = torch.zeros(m, dtype=t.dtype)
        pad[:t.numel()] = t
        outs = [torch.empty(m, dtype=t.dtype) for _ in range(world)]
        dist.all_gather(outs, pad)
        res = [o[:int(n)] for o, n in zip(outs, sizes)]
        if corrupt and rank == 1:
            res[0] = res[0] + 1
        return res

    fake = types.SimpleNamespace(ops=types.SimpleNamespace(_Test_NCCLTensorAllGather=allgather))
    args = bench.parse(["--check-batches", "0"])
    try:
        res = bench.multi_rank_self_check(fake, dist, None, None, None, None, [5], args, None,
                                          rank, world, torch.device("cpu"), True)
        verdict = res["allgather"]
    except SystemExit as e:
        verdict = f"exit {e.code}"
    with open(f"{out}/r{rank}.txt", "w") as f:
        f.write(verdict)
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_multi_rank_self_check_verdict(tmp_path, corrupt):
    """Rank-dependent payload lengths all-gathered and checked on every rank; one bad payload
    on one rank makes every rank exit non-zero (the verdict is all-reduced)."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_selfcheck_worker, args=(2, port, corrupt, str(tmp_path)), nprocs=2, join=True)
    got = [open(tmp_path / f"r{r}.txt").read() for r in range(2)]
    assert got == (["exit 1", "exit 1"] if corrupt else ["ok", "ok"])


def test_compare_batches_counts_mismatches():
    b = [(torch.arange(3), torch.arange(5), torch.arange(4), torch.arange(4))]
    x, y = torch.ones(5, 2), torch.arange(3)
    good = [(b, x, y)]
    assert bench.compare_batches(good, [(b, x.clone(), y.clone())]) == 0
    b2 = [(torch.arange(3), torch.arange(5), torch.arange(4), torch.tensor([0, 1, 2, 4]))]
    assert bench.compare_batches(good, [(b2, x, y)]) == 1
    assert bench.compare_batches(good, [(b, x + 1, y)]) == 1
    assert bench.compare_batches(good, []) == 1


def test_secondary_papers_bias_record_only_for_the_default_single_gpu_run():
    """The default N = 1 run adds configs[3] (papers-like graph, degree-weighted biased sampler,
    d = 128) as a nested record; any other workload, N > 1, or --secondary none does not."""
    sec = bench.secondary_workload(bench.parse([]), 1)
    assert sec["scale"] == 27 and sec["ef"] == 12 and sec["dim"] == 128 and sec["bias"]
    assert sec["secondary"] == "none" and sec["mode"] == "replicated"
    assert bench.secondary_workload(bench.parse([]), 2) is None
    assert bench.secondary_workload(bench.parse(["--bias"]), 1) is None
    assert bench.secondary_workload(bench.parse(["--secondary", "none"]), 1) is None
    assert bench.secondary_workload(bench.parse(["--scale", "17", "--secondary", "papers_bias"]),
                                    1) is not None
    a2 = bench.parse([])
    for k, v in sec.items():
        setattr(a2, k, v)
    assert bench.baseline_config(a2, "replicated", None).startswith("configs[3]")
    assert bench.baseline_config(bench.parse([]), "replicated", None) == "configs[1]"
    assert bench.baseline_config(bench.parse([]), "hot-shard", None) == "configs[2]"


def test_step_floor_counts_bytes_and_draws():
    """bench.step_floor: SURVEY 8(d) bytes per hop + gather/label bytes, and the Philox work of
    the VALU-bound kernels (uniform: deg - k per row with deg > k; biased: deg per such row plus
    the boot sample of rows above 1024)."""
    import numpy as np
    import torch
    import bench
    indptr = torch.tensor([0, 20, 23, 2023, 2030])  # degrees 20, 3, 2000, 7
    seeds = torch.tensor([0, 1, 2, 3])
    fr = torch.arange(10)
    r = torch.zeros(12, dtype=torch.int64)
    blocks = [(seeds, fr, r, r)]
    f = bench.step_floor([blocks], indptr, [5], False, 4, 1.0)
    S, nnz, Sp = 4, 12, 10
    sample_b = 8 * S + 16 * S + 8 * nnz + 16 * nnz + 8 * (S + nnz) + 8 * Sp + 16 * nnz
    assert f["hbm_bytes_per_step"] == sample_b + 10 * (2 * 4 * 4 + 8) + 24 * 4
    assert f["philox_draws_per_step"] == (20 - 5) + (2000 - 5) + (7 - 5)
    assert np.isclose(f["valu_floor_us"], f["philox_draws_per_step"] * bench.UNIFORM_INSTR_PER_DRAW
                      / bench.PEAK_WAVE_INSTR_PER_S * 1e6)
    assert np.isclose(f["valu_at_measured_rate_us"],
                      f["philox_draws_per_step"] / bench.UNIFORM_DRAWS_PER_S * 1e6)
    assert f["max_us"] == max(f["hbm_floor_us"], f["valu_floor_us"])
    fb = bench.step_floor([blocks], indptr, [5], True, 4, 1.0)
    assert fb["philox_draws_per_step"] == 20 + 2000 + 7 + 2000  # + boot sample of the hub row
    assert fb["hbm_bytes_per_step"] == f["hbm_bytes_per_step"] + 4 * (20 + 2000 + 7)
