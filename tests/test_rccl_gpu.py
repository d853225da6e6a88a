"""The library's RCCL transport on a tested path: a world-1 communicator (one GPU holds one
RCCL rank) built by create_communicator, then the barrier, TensorP2PServer, the all-gather and
services under it (tests/rccl_worker.py, a fresh process: the communicator is process-global).
The multi-rank data path is covered by tests/test_multirank_gpu.py over the host transport."""
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


def _run_worker(*extra):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r.json")
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        rc = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py"), out, *extra],
                            env=env, timeout=180).returncode
        assert rc == 0
        return json.load(open(out))


@pytest.fixture(scope="module")
def res():
    return _run_worker()


@pytest.fixture(scope="module")
def res_self():
    return _run_worker("self")


def test_rccl_grouped_send_recv_self_exchange(res_self):
    """The grouped ncclSend / ncclRecv all-gather (nccl_context.cc:52-112) executed on the GPU:
    with the own rank as a peer, the world-1 communicator moves every payload through RCCL."""
    assert res_self["world"] == 1
    assert res_self["sizes"] == [12345]
    assert res_self["bytes_equal"] and res_self["bytes_nonzero"] > 3 * (1 << 20) * 0.99
    assert res_self["allgather"] == [[x + 0.5 for x in range(7)]]
    assert res_self["feature_kat"] == [[float(x) for x in range(b, b + 10)]
                                       for b in (0, 30, 50, 70)]
    assert res_self["barrier_rc"] == 0


def test_rccl_communicator_world1(res):
    assert res["world"] == 1 and res["rank"] == 0
    assert res["barrier_rc"] == 0 and res["barrier_rc_end"] == 0


def test_rccl_p2p_server_and_allgather(res):
    # tests/test_p2p_server.py: cache [0, 3] -> sub-indptr [0, 4, 4]
    assert res["p2p_view"] == [0, 4, 4] and res["p2p_local"] == [0, 4, 4]
    assert res["allgather"] == [[0.0, 1.0, 2.0, 3.0, 4.0]]


def test_rccl_services(res):
    exp = [[float(x) for x in range(b, b + 10)] for b in (0, 30, 50, 70)]
    assert res["feature_kat"] == exp
    ip = np.array([0, 4, 5, 5, 5, 5, 10, 10, 10, 10, 10, 10], dtype=np.int64)
    ix = np.arange(1, 11, dtype=np.int64)
    want = O.node_classification_sample(np.array([0, 3, 5]), ip, ix, [2, 2], False,
                                         O.launch_seeds(99, 2))
    for (gf, gr, gc), (_, ef, er, ec) in zip(res["sample"], want):
        assert gf == ef.tolist() and gr == er.tolist() and gc == ec.tolist()
