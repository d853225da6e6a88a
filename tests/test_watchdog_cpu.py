"""Bounded failure of a stalled multi-rank setup (DistGNN.dist.SetupWatchdog, used by bench.py
at N > 1): with one rank of a gloo world of two withholding a collective, BOTH ranks exit
non-zero within the bound, naming their step; a setup that completes exits 0."""
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(mode, bound):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "watchdog_worker.py"),
                                       mode, str(bound)], env=env, stderr=subprocess.PIPE,
                                      text=True))
    out = []
    for p in procs:
        try:
            _, err = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            p.kill()
            _, err = p.communicate()
        out.append((p.returncode, err))
    return out, time.time() - t0


def test_withheld_collective_ends_both_ranks_within_the_bound():
    bound = 4.0
    out, el = _run("withhold", bound)
    assert [rc for rc, _ in out] == [3, 3], out
    assert "step 'barrier'" in out[0][1]
    assert "step 'rank 1 work before the barrier'" in out[1][1]
    # rendezvous + bound + the poll interval, far below the 120 s the worker would stall
    assert el < bound + 30, el


def test_completed_setup_exits_cleanly():
    out, _ = _run("ok", 20.0)
    assert [rc for rc, _ in out] == [0, 0], out
