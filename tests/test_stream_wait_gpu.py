"""The C-ABI cross-stream wait (dgs_stream_wait, used by PrefetchLoader in both directions):
a batch stream that waits for the caller's stream must see every write the caller enqueued
before the wait, even when that work is still running (a long spin kernel ahead of it), and
with the caller on the default (null) stream or on a pool stream.  The event is per thread and
re-recorded at once by the next wait, so the waits are issued back to back."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


@pytest.mark.parametrize("caller", ["default", "pool"])
def test_wait_orders_after_pending_work(dgs, caller):
    dev = torch.device("cuda", 0)
    c_stream = torch.cuda.default_stream(dev) if caller == "default" else torch.cuda.Stream(dev)
    b_streams = [torch.cuda.Stream(dev) for _ in range(3)]
    n = 1 << 20
    bufs = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in b_streams]
    outs = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in b_streams]
    torch.cuda.synchronize()
    bad = 0
    for it in range(1, 41):
        with torch.cuda.stream(c_stream):
            for i, buf in enumerate(bufs):
                torch.cuda._sleep(200_000)  # keeps the fill below pending for a while
                buf.fill_(it * 10 + i)
        for i, (bs, buf, out) in enumerate(zip(b_streams, bufs, outs)):
            dgs.ops._stream_wait(c_stream.cuda_stream, bs.cuda_stream)
            with torch.cuda.stream(bs):
                out.copy_(buf)
        torch.cuda.synchronize()
        for i, out in enumerate(outs):
            bad += int((out != it * 10 + i).sum())
    assert bad == 0
