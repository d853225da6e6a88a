"""Pipelined mini-batch preparation (ADDITIVE).

The reference loop (example/graphsage/node_classification.py:219-229) makes its three calls
back to back on one stream: sample, feature gather, label gather.  A sample call is a chain of
small dependent kernels, so one batch leaves most of the GPU idle.  A multi-hop sample needs no
host synchronisation until its sizes are read (grids are sized from host-side bounds), so
PrefetchLoader enqueues the next `depth - 1` batches' calls on their own streams before it
waits for the current one.  One thread, one sampler and one feature server: the sampler keeps a
sampling context per stream over the shared graph.
"""
import collections
import os
import threading

import torch

import dgs

__all__ = ["PrefetchLoader"]

# Streams are reused by every loader on a device: the sampler keeps one sampling context
# (scratch, relabel tables: 16 B per node) per stream for its lifetime, and a context's first
# use allocates it.
_STREAMS = {}
# DGS_PREFETCH_SYNC=1: issue each batch's launches on the caller's thread (experiments)
_HOST_ASYNC = os.environ.get("DGS_PREFETCH_SYNC", "0") != "1"
_STREAMS_LOCK = threading.Lock()


def _worker_streams(device, n):
    with _STREAMS_LOCK:
        pool = _STREAMS.setdefault(device, [])
        while len(pool) < n:
            pool.append(torch.cuda.Stream(device=device))
        return pool[:n]



class PrefetchLoader:
    """Yields, in batch order, `(blocks, x, y)` for each seed batch of `seeds_iter`:

    - blocks = sampler._CAPI_sample_node_classifiction(seeds, fan_out, replace),
    - x = server._CAPI_get_feature(blocks[-1][1]), or None without a server,
    - y = dgs.ops._CAPI_cuda_index_select(labels, seeds), or None without labels.

    Up to `depth` batches are in flight, batch i on stream i mod depth.  Every tensor handed out
    is ready on the caller's current stream when __next__ returns (that stream waits for the
    batch's stream; the host does not block on it).  Each batch's per-hop launch seeds are
    drawn from the global engine in batch order, so the output is exactly that of the
    sequential loop after the same dgs.ops._CAPI_set_random_seed.
    """

    def __init__(self, sampler, seeds_iter, fan_out, replace=False, server=None, labels=None,
                 depth=2, device=None):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.sampler, self.server, self.labels = sampler, server, labels
        self.fan_out, self.replace = list(fan_out), bool(replace)
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self._seeds = iter(seeds_iter)
        self._exhausted = False
        self._streams = _worker_streams(self.device, depth)
        # reusable cross-stream events: caller -> batch stream, batch stream -> caller (one
        # gather stream per batch stream: more streams than the process's hardware queues
        # would serialise them)
        self._ev_submit = [torch.cuda.Event() for _ in range(depth)]
        self._ev_done = torch.cuda.Event()
        self._inflight = collections.deque()
        self._n = 0

    def _submit(self):
        try:
            seeds = next(self._seeds)
        except StopIteration:
            self._exhausted = True
            return
        w = self._n % len(self._streams)
        st = self._streams[w]
        self._n += 1
        # the seeds (and any memory the caller's stream recycled) come from the caller's stream
        ev = self._ev_submit[w]
        ev.record(torch.cuda.current_stream(self.device))
        st.wait_event(ev)
        seeds.record_stream(st)
        launch_seeds = dgs.ops.draw_launch_seeds(len(self.fan_out))
        with torch.cuda.stream(st):
            y = None
            if self.labels is not None:  # depends on the seeds only: issued first
                y = dgs.ops._CAPI_cuda_index_select(self.labels, seeds)
            # the stream is not touched again before result(): the sampler's launcher thread
            # may issue the launches
            pending = self.sampler._sample_begin(seeds, self.fan_out, self.replace,
                                                 launch_seeds, host_async=_HOST_ASYNC)
        self._inflight.append((pending, y, st))

    def __iter__(self):
        return self

    def __next__(self):
        while not self._exhausted and len(self._inflight) < len(self._streams):
            self._submit()
        if not self._inflight:
            raise StopIteration
        pending, y, st = self._inflight.popleft()
        try:
            with torch.cuda.stream(st):
                blocks = pending.result()
        except BaseException:
            self.close()
            raise
        x = None
        if self.server is not None:
            with torch.cuda.stream(st):
                x = self.server._CAPI_get_feature(blocks[-1][1])
        cur = torch.cuda.current_stream(self.device)
        self._ev_done.record(st)
        cur.wait_event(self._ev_done)
        # the caller's stream now uses memory allocated on the batch's streams: with int64 ids
        # every block tensor but the caller's seeds is a view of one buffer
        if blocks[-1][1].dtype == torch.int64:
            blocks[-1][1].record_stream(cur)
        else:
            for b in blocks:
                for t in b[1:]:
                    t.record_stream(cur)
        for t in (x, y):
            if t is not None:
                t.record_stream(cur)
        return blocks, x, y

    def close(self):
        """Ends the calls still in flight (a stream takes a new call only after its last one
        has ended); their results are dropped."""
        while self._inflight:
            pending, _, st = self._inflight.popleft()
            try:
                with torch.cuda.stream(st):
                    pending.result()
            except Exception:
                pass
        self._exhausted = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
