"""Round 4: the root cause of the round-3 N = 2 corruption, pinned in one process.

Round 3 saw, with two bench processes on one GPU, a hop-0 neighbour id that held two packed f32
feature words (and once a GPU fault in the relabel pass).  The loader orders each batch stream B
after the caller's stream C with dgs_sampler_sample_begin_after(wait_for = C).  That entry point
tested the *handle* ("wait when non-NULL"), and torch's default current stream -- the caller's
stream in the bench -- is the null stream, handle 0: B never waited for C.  Rounds 2-3 allocated
the sample-output buffer from C's pool, so a later batch's buffer could be carved from an x
whose feature gather was still queued on C, and that gather then wrote feature rows over the
sampler's output.  One process rarely shows it (C's gathers finish before B's kernels reach the
memory); two processes sharing the GPU delay each other's kernels enough.  Now a flag
(DGS_SAMPLE_WAIT) requests the wait and NULL is a stream like any other.

These tests stall C with spin kernels so that the missing wait would be seen every time:
- seeds written on C behind a stall must be the seeds the sampler reads (caller on the null
  stream and on a pool stream; the raw entry point and PrefetchLoader);
- the round-2/3 loader ordering (buffers from C's pool) with C stalled in front of each batch's
  C-side work: the allocator must really hand a later batch a buffer overlapping a dropped x
  whose C-side writes are still queued, and every batch must stay bit-exact.  The C-side write
  is a pattern fill of x, not the feature gather, so that a regression shows as a mismatch or a
  range-check error instead of a gather reading overwritten frontier ids (a GPU fault: that is
  what this test did against the unfixed library on the round-4 box)."""
import collections

import pytest
import torch

pytestmark = pytest.mark.gpu

STALL = 400_000  # torch.cuda._sleep cycles (~0.2 ms): longer than one small batch's kernels


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


def _services(dgs, dim):
    from DistGNN.dataloading.synthetic import rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(13, 12, seed=20261015)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(n), 0)
    feats = torch.randn(n, dim, generator=torch.Generator().manual_seed(4))
    server = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(n), 0)
    labels = torch.randint(0, 40, (n,), generator=torch.Generator().manual_seed(0)).cuda()
    return sampler, server, labels, n


def _batches(n, nb, bsz):
    g = torch.Generator().manual_seed(12)
    return [torch.randint(0, n, (bsz,), generator=g).cuda() for _ in range(nb)]


def _same_blocks(a, b):
    return len(a) == len(b) and all(torch.equal(u, v) for ta, tb in zip(a, b)
                                    for u, v in zip(ta, tb))


@pytest.mark.parametrize("caller", ["null", "pool"])
@pytest.mark.parametrize("host_async", [False, True])
def test_batch_stream_waits_for_seeds_written_on_caller_stream(dgs, caller, host_async):
    """dgs_sampler_sample_begin_after(wait_for = C, DGS_SAMPLE_WAIT): seeds that C writes behind
    a long spin kernel are the seeds the batch stream samples, also when C is the null stream
    (handle 0: the round-2/3 entry point skipped the wait for it)."""
    sampler, _, _, n = _services(dgs, dim=4)
    fan_out = [15, 10, 5]
    final = _batches(n, 1, 256)[0]
    dgs.ops._CAPI_set_random_seed(3)
    exp = sampler._CAPI_sample_node_classifiction(final, fan_out, False)
    c = torch.cuda.default_stream() if caller == "null" else torch.cuda.Stream()
    b = torch.cuda.Stream()
    assert (c.cuda_stream == 0) == (caller == "null")
    for _ in range(3):
        seeds = torch.zeros_like(final)  # node 0 until C overwrites it
        torch.cuda.synchronize()
        with torch.cuda.stream(c):
            torch.cuda._sleep(4 * STALL)
            seeds.copy_(final)
            prep = sampler._prepare(seeds, fan_out, packed=True)
        dgs.ops._CAPI_set_random_seed(3)
        pending = sampler._begin_prepared(seeds, prep, False, None, host_async, b.cuda_stream,
                                          wait_for=c.cuda_stream)
        got = pending.result()
        torch.cuda.synchronize()
        assert _same_blocks(got, exp)


def test_loader_waits_for_seeds_written_on_caller_stream(dgs):
    """The same through PrefetchLoader on the default (null) stream: every batch's seeds are
    written on the caller's stream behind a spin kernel just before the loader submits it."""
    from DistGNN.dataloading import PrefetchLoader
    sampler, server, labels, n = _services(dgs, dim=8)
    fan_out = [10, 5]
    final = _batches(n, 6, 128)
    dgs.ops._CAPI_set_random_seed(8)
    exp = [sampler._CAPI_sample_node_classifiction(s, fan_out, False) for s in final]

    def late_seeds():
        for s in final:
            t = torch.zeros_like(s)
            torch.cuda._sleep(2 * STALL)
            t.copy_(s)
            yield t

    dgs.ops._CAPI_set_random_seed(8)
    got = [blocks for blocks, _, _ in PrefetchLoader(sampler, late_seeds(), fan_out,
                                                     server=server, labels=labels, depth=3)]
    torch.cuda.synchronize()
    assert len(got) == len(exp) and all(_same_blocks(g, e) for g, e in zip(got, exp))


class _OldOrderLoader:
    """The round-2/3 PrefetchLoader ordering (before commit c4a24d2: sample-output buffers from
    the caller's stream pool, no record_stream; B waits for C after the allocations), with the
    C-side work of each handed-out batch replaced by a stall and a pattern fill of x."""

    def __init__(self, dgs, sampler, batches, fan_out, depth, stall_c):
        self.dgs, self.sampler, self.fan_out, self.stall_c = dgs, sampler, fan_out, stall_c
        self.streams = [torch.cuda.Stream() for _ in range(depth)]
        self.it = iter(batches)
        self.inflight = collections.deque()
        self.n = 0
        self.buf_ranges = []  # (batch, ptr, bytes) of every sample-output buffer

    def _submit(self):
        s = next(self.it, None)
        if s is None:
            return False
        w = self.n % len(self.streams)
        b = self.streams[w]
        cur = torch.cuda.current_stream().cuda_stream
        s.record_stream(b)
        prep = self.sampler._prepare(s, self.fan_out, packed=True)  # buffer from C's pool
        buf = prep[5]
        self.buf_ranges.append((self.n, buf.data_ptr(), buf.numel() * 8))
        pending = self.sampler._begin_prepared(s, prep, False, None, True, b.cuda_stream,
                                               wait_for=cur)
        self.inflight.append((pending, w))
        self.n += 1
        return True

    def __iter__(self):
        while True:
            while len(self.inflight) < len(self.streams) and self._submit():
                pass
            if not self.inflight:
                return
            pending, w = self.inflight.popleft()
            blocks = pending.result(cast=False)
            cur = torch.cuda.current_stream().cuda_stream
            self.dgs.ops._stream_wait(self.streams[w].cuda_stream, cur)  # C after B
            x = torch.empty((blocks[-1][1].numel(), 256), dtype=torch.float32, device="cuda")
            torch.cuda._sleep(self.stall_c)  # the write below runs late on C
            x.fill_(3.3961e38)  # bits 0x7F7F7F7F: as an int64 id, far outside [0, N)
            yield blocks, x


def test_old_allocation_order_with_the_wait_is_sound(dgs):
    sampler, _, _, n = _services(dgs, dim=4)
    fan_out = [15, 10, 5]
    batches = _batches(n, nb=40, bsz=128)
    dgs.ops._CAPI_set_random_seed(91)
    exp = [sampler._CAPI_sample_node_classifiction(s, fan_out, False) for s in batches]
    torch.cuda.synchronize()
    dgs.ops._CAPI_set_random_seed(91)
    ld = _OldOrderLoader(dgs, sampler, batches, fan_out, depth=3, stall_c=STALL)
    got, x_ranges = [], []
    for i, (blocks, x) in enumerate(ld):
        x_ranges.append((i, x.data_ptr(), x.numel() * 4))
        got.append(blocks)  # held: the next buffers must come from the dropped x blocks
        del x, blocks
    torch.cuda.synchronize()
    # the window is exercised: later buffers overlap earlier x whose fill was still queued
    hits = sum(1 for j, bp, bb in ld.buf_ranges for i, xp, xb in x_ranges
               if i < j and bp < xp + xb and xp < bp + bb)
    assert hits > 0
    assert len(got) == len(exp) and all(_same_blocks(g, e) for g, e in zip(got, exp))


def test_current_loader_under_stalls(dgs):
    """PrefetchLoader as shipped (outputs from the batch stream's pool), the caller's stream
    stalled behind every batch and x dropped at once: bit-exact blocks, features and labels."""
    from DistGNN.dataloading import PrefetchLoader
    fan_out = [15, 10, 5]
    sampler, server, labels, n = _services(dgs, dim=256)
    batches = _batches(n, nb=40, bsz=128)
    dgs.ops._CAPI_set_random_seed(93)
    exp = []
    for s in batches:
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        exp.append((blocks, server._CAPI_get_feature(blocks[-1][1]), labels[s]))
    torch.cuda.synchronize()
    dgs.ops._CAPI_set_random_seed(93)
    got = []
    for blocks, x, y in PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                                       depth=3):
        torch.cuda._sleep(STALL)  # the caller's stream runs late behind every batch
        got.append((blocks, x.clone(), y))
        del x
    torch.cuda.synchronize()
    for (gb, gx, gy), (eb, ex, ey) in zip(got, exp):
        assert _same_blocks(gb, eb) and torch.equal(gx, ex) and torch.equal(gy, ey)
    assert len(got) == len(exp)
