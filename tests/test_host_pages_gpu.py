"""Host pages shared between the library's host state and torch's own pageable copies
(round 6, DESIGN.md section 3: the three hipErrorIllegalAddress records of rounds 4-5 all
surfaced in torch's pageable host copies).

The layout is built deterministically inside one pageable numpy buffer, whose views become
torch tensors with their own storages (torch.from_numpy of a view): a pinned region A whose
first and last pages it shares with the pageable neighbours B (after it) and C (before it);
then services over pageable neighbours of the same pages.  B and C are copied host-to-device
and device-to-host -- the copies HIP performs by pinning the caller's pages for the transfer --
before, during and after A's pin and the services' lives, and every copy is checked byte for
byte.  A separate case pins, unpins and frees a buffer, then copies through a fresh allocation
of the same size (which the allocator may place at the same addresses)."""
import gc

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
PAGE = 4096
MB = 1 << 20


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    torch.cuda.set_device(0)
    return _dgs


def _fill(a, seed):
    a[:] = np.random.default_rng(seed).integers(0, 256, a.size, dtype=np.uint8)


def _round_trip(t, seed):
    """t (a pageable uint8 tensor) -> device -> back into t; both directions checked."""
    want = t.clone()
    d = t.cuda()
    assert torch.equal(d.cpu(), want)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    new = torch.randint(0, 256, (t.numel(),), generator=g, device="cuda", dtype=torch.uint8)
    t.copy_(new)  # device to pageable host
    assert torch.equal(t, new.cpu())
    t.copy_(want)


def _regs_in(lo, hi, dgs):
    return [(r["base"], r["bytes"]) for r in dgs.ops._host_registrations()
            if lo <= r["base"] < hi]


def test_copies_of_pages_shared_with_a_pin_and_services(dgs):
    buf = np.zeros(96 * MB, dtype=np.uint8)
    lo, hi = buf.ctypes.data, buf.ctypes.data + buf.size
    # region offsets: neither end of A on a page boundary (A shares a page with B and with C)
    page0 = (-buf.ctypes.data) % PAGE
    c0 = page0 + 5 * PAGE + 0x10
    a0 = page0 + 9 * PAGE + 0x40
    a1 = a0 + 6 * MB + 0x123
    b1 = a1 + 24 * MB + 77
    assert a0 // PAGE * PAGE < a0 and a1 % PAGE and b1 < buf.size
    _fill(buf, 1)
    A = torch.from_numpy(buf[a0:a1])
    B = torch.from_numpy(buf[a1:b1])
    C = torch.from_numpy(buf[c0:a0])
    a_want = A.clone()
    for i, t in enumerate((B, C)):
        _round_trip(t, 10 + i)

    # A pinned in place (pin_memory.cc:7-12): its end pages hold B's and C's first / last bytes
    dgs.ops._CAPI_tensor_pin_memory(A)
    assert _regs_in(lo, hi, dgs) == [(A.data_ptr(), A.numel())]
    for i, t in enumerate((B, C)):
        _round_trip(t, 20 + i)
    # A read through its mapping while B / C are copied
    rows = A.numel() // 64
    a2 = A[: rows * 64].view(rows, 64)
    q = np.random.default_rng(3).integers(0, rows, 8192)
    m0 = dgs.ops._host_memory_state()["mirrors"]
    fs = dgs.classes.P2PCacheFeatureServer(a2, torch.tensor([0, 5]), 0)
    assert dgs.ops._host_memory_state()["mirrors"] == m0  # in place, on the pin
    _round_trip(B, 30)
    x = fs._CAPI_get_feature(torch.from_numpy(q).cuda())
    assert np.array_equal(x.cpu().numpy(), O.index_select(a2.numpy(), q))
    y = dgs.ops._CAPI_cuda_index_select(a2.view(torch.int32), torch.from_numpy(q).cuda())
    assert torch.equal(y.cpu(), a2.view(torch.int32)[torch.from_numpy(q)])
    dgs.ops._CAPI_tensor_unpin_memory(A)
    _round_trip(C, 31)
    del fs, x, y
    gc.collect()
    torch.cuda.synchronize()
    assert _regs_in(lo, hi, dgs) == []
    assert torch.equal(A, a_want)
    for i, t in enumerate((B, C)):
        _round_trip(t, 40 + i)

    # services over pageable B (partly cached: a pinned mirror, B itself is never registered)
    # while B's neighbours and B are copied
    rows_b = B.numel() // 96
    b2 = B[: rows_b * 96].view(rows_b, 96)
    before = dgs.ops._host_memory_state()
    fsb = dgs.classes.P2PCacheFeatureServer(b2, torch.arange(0, rows_b, 7), 0)
    st = dgs.ops._host_memory_state()
    assert st["registrations"] == before["registrations"]
    assert st["mirrors"] == before["mirrors"] + 1
    assert not B.is_pinned()
    qb = np.random.default_rng(4).integers(0, rows_b, 16384)
    want = O.index_select(b2.numpy(), qb)
    _round_trip(C, 50)
    assert np.array_equal(fsb._CAPI_get_feature(torch.from_numpy(qb).cuda()).cpu().numpy(), want)
    _round_trip(A, 51)
    del fsb
    gc.collect()
    assert dgs.ops._host_memory_state() == before
    _round_trip(B, 52)


def test_copies_through_a_reused_range_after_unpin(dgs):
    """pin -> unpin -> free -> a fresh allocation of the same size (the allocator may hand back
    the same addresses) -> pageable copies both ways through it, exact."""
    n = 64 * MB
    for rep in range(3):
        x = torch.empty(n, dtype=torch.uint8)
        x.fill_(rep + 1)
        dgs.ops._CAPI_tensor_pin_memory(x)
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        d.copy_(x)  # from the pinned range
        assert int(d[::4096].sum()) == (rep + 1) * (n // 4096)
        dgs.ops._CAPI_tensor_unpin_memory(x)
        assert _regs_in(x.data_ptr(), x.data_ptr() + n, dgs) == []
        del x
        gc.collect()
        y = torch.empty(n, dtype=torch.uint8)
        y.copy_(d)  # device to pageable host, possibly at the old addresses
        assert torch.equal(y[::4099], torch.full_like(y[::4099], rep + 1))
        y.fill_(7)
        d.copy_(y)
        assert int(d[::4096].sum()) == 7 * (n // 4096)
        del y, d
    dgs.ops._check_async_errors()
