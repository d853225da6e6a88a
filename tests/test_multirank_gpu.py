"""Two ranks sharing cuda:0 exercise the multi-rank path: IPC export / import of every cache
block, cache-list all-gathers, node/feature tables with peer entries, one-sided peer reads.
Results must equal the single-process oracle (P2P-cached output == uncached output)."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def results():
    world = 2
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        procs = []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), LOCAL_RANK="0")
            procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"),
                                           os.path.join(td, f"r{r}.json")], env=env))
        rcs = [p.wait(timeout=240) for p in procs]
        assert rcs == [0] * world, rcs
        return [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]


def test_world_and_allgather(results):
    for r, res in enumerate(results):
        assert res["world"] == 2 and res["local_rank"] == r
        assert res["allgather"] == [[0.0, 0.0], [1.0, 1.0, 1.0]]


def test_p2p_server_kat(results):
    # tests/test_p2p_server.py: rank0 caches [0,3] -> [0,4,4]; rank1 [3,5] -> [0,0,5]
    for res in results:
        assert res["p2p_views"] == [[0, 4, 4], [0, 0, 5]]


def test_feature_server_kat(results):
    exp = [[float(x) for x in range(b, b + 10)] for b in (0, 30, 50, 70)]
    for res in results:
        assert res["feature_kat"] == exp


def test_sharded_sampler_matches_oracle(results):
    rng = np.random.default_rng(0)
    n = 600
    degs = rng.integers(0, 70, n)
    degs[:4] = [0, 3000, 1500, 20]
    ip = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    ix = rng.integers(0, n, int(ip[-1])).astype(np.int64)
    probs = (rng.random(ix.size) + 0.05).astype(np.float32)
    for res in results:
        for bias in (0, 1):
            got = res[f"sample_bias{bias}"]
            exp = O.node_classification_sample(np.array(got["seeds"]), ip, ix, [10, 5], False,
                                               O.launch_seeds(777, 2),
                                               probs=probs if bias else None)
            for (gf, gr, gc), (_, ef, er, ec) in zip(got["hops"], exp):
                assert gf == ef.tolist() and gr == er.tolist() and gc == ec.tolist()


def test_cache_map_local_priority(results):
    for r, res in enumerate(results):
        key, idx, devid = res["map_bias0"]
        assert key == list(range(600))
        assert devid == [v % 2 for v in range(600)]
        assert idx == [v // 2 for v in range(600)]


def test_reference_cache_hashmap_layout(results):
    """_CAPI_get_local_cache_hashmap_tensors: the reference's open-addressing map built from
    both ranks' lists (hashmap.cu:15-77): capacity 2 * _UpPower(600), the key set, and every
    node's (idx, devid) reached by the reference's probe sequence (SearchForPos)."""
    for r, res in enumerate(results):
        key, idx, devid = (np.array(a) for a in res["refmap_bias0"])
        assert len(key) == O.cache_hashmap_dir_size(600) == 2048
        assert sorted(key[key >= 0].tolist()) == list(range(600))
        assert (idx[key < 0] == -1).all() and (devid[key < 0] == -1).all()
        for v in range(600):
            pos = O.cache_hashmap_find(key, v)
            assert pos >= 0 and idx[pos] == v // 2 and devid[pos] == v % 2


def test_sharded_gather(results):
    assert all(res["gather_ok"] for res in results)
    # v mod 2 shard -> strided layout (peer rows through the IPC-mapped block, no table)
    assert all(res["gather_layout"] == 1 for res in results)


def _setup_failure(mode, extra_env):
    world = 2
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        procs = []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), LOCAL_RANK="0", **extra_env)
            procs.append(subprocess.Popen([sys.executable,
                                           os.path.join(HERE, "ipc_fail_worker.py"),
                                           os.path.join(td, f"r{r}.txt"), mode], env=env))
        rcs = [p.wait(timeout=120) for p in procs]
        assert rcs == [0] * world, rcs
        return [open(os.path.join(td, f"r{r}.txt")).read().splitlines() for r in range(world)]


def test_failed_export_raises_on_every_rank():
    """A rank whose hipIpcGetMemHandle fails still takes part in the handle exchange, and every
    rank raises naming it (services.cpp P2PServer::share), instead of its peers waiting in the
    collective.  Both the TensorP2PServer constructor and an adopted service block
    (P2PCacheFeatureServer) are checked; the process group works afterwards."""
    for msgs in _setup_failure("export", {"DGS_TEST_IPC_EXPORT_FAIL": "1"}):
        assert len(msgs) == 2, msgs
        for m in msgs:
            assert "rank 1 could not export its block" in m, m


def test_bad_argument_on_one_rank_raises_on_every_rank():
    """One rank's out-of-range cache id (the services' first, local checks) is made collective
    (Comm::check_all): every rank raises naming rank 1, the failing rank with its own error,
    and no rank waits in the cache-list exchange."""
    r0, r1 = _setup_failure("args", {})
    assert r0[-1] == r1[-1] == "after: ok", (r0, r1)
    for m in r0[:-1]:
        assert "failed on rank(s) 1" in m and "this rank's part succeeded" in m, m
    for m in r1[:-1]:
        assert "failed on rank(s) 1" in m and "outside" in m, m


def test_build_failure_on_one_rank_raises_on_every_rank():
    """A rank whose cache build fails (host sources, sub-CSR or feature block; DGS_TEST_BUILD_FAIL
    test hook) raises with every other rank before the blocks are exchanged, and a second
    service can be built collectively afterwards (the process group and library state are
    usable)."""
    r0, r1 = _setup_failure("build", {"DGS_TEST_BUILD_FAIL": "1"})
    assert r0[-1] == r1[-1] == "after: ok", (r0, r1)
    for m in r0[:-1]:
        assert "building the cache failed on rank(s) 1" in m and "succeeded" in m, m
    for m in r1[:-1]:
        assert "building the cache failed on rank(s) 1" in m and "test hook" in m, m


def test_random_cache_placements_match_oracle():
    """tools/mr_sweep.py for a short while: 2 ranks, a new random graph per case whose services
    both ranks build with a random cache placement (each node cached by no rank, one or both),
    every rank's blocks against the oracle and its features against a host index."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(os.path.dirname(HERE), "tools", "mr_sweep.py"), "--seconds", "15",
           "--seed", "11"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "0 mismatches" in p.stdout, p.stdout[-2000:]
