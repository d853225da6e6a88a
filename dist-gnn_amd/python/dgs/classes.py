"""dgs.classes -- mirror of the reference's `m_classes` submodule (src/pybind.cc:19-45):
P2PCacheSampler, P2PCacheFeatureServer and TensorP2PServer with the same constructor
arguments, method names (including the `_CAPI_sample_node_classifiction` spelling) and
return shapes.  State lives in libdgs_amd.so; this layer only moves tensors across the C ABI.
"""
import ctypes

import torch

from ._lib import c_i64, c_vp, check, i64_array, lib, stream_ptr, vp_array
from ._util import as_i64, check_cpu, check_cuda, device_view, ptr, row_bytes


def _host_i64(t, name):
    check_cpu(t, name)
    return as_i64(t, name)


class TensorP2PServer:
    """tensor_p2p_cache.{h,cc}: a CUDA tensor copied into a library block and shared with
    every rank through HIP IPC (collective when world_size > 1)."""

    def __init__(self, tensor):
        check_cuda(tensor, "tensor")
        t = tensor.contiguous()
        if t.dim() == 0 or t.shape[0] <= 0:
            raise RuntimeError("TensorP2PServer needs at least one item")
        self._shape = tuple(t.shape)
        self._dtype = t.dtype
        self._stride, item_bytes = row_bytes(t)
        h = c_vp()
        check(lib.dgs_p2p_server_create(ptr(t), t.shape[0], item_bytes, ctypes.byref(h)))
        self._h = h

    def _device(self, rank):
        p, n = c_vp(), c_i64()
        check(lib.dgs_p2p_server_device_ptr(self._h, int(rank), ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def _CAPI_get_device_tensor(self, device_id):
        """1-D view of items * stride elements (tensor_p2p_cache.cc:126-132)."""
        p, n = self._device(device_id)
        return device_view(p, (n * self._stride,), self._dtype, self)

    def _CAPI_get_local_device_tensor(self):
        p, _ = self._device(lib.dgs_get_local_rank())
        return device_view(p, self._shape, self._dtype, self)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.dgs_p2p_server_destroy(h)
            self._h = None


def plan_ptrs(base, caps):
    """Pointer arrays of the per-hop (frontier, row, col) buffers laid out back to back."""
    fr_p, row_p, col_p, off = [], [], [], 0
    for f, e in caps:
        fr_p.append(base + 8 * off)
        row_p.append(base + 8 * (off + f))
        col_p.append(base + 8 * (off + f + e))
        off += f + 2 * e
    return vp_array(fr_p), vp_array(row_p), vp_array(col_p)


class P2PCacheSampler:
    """sampler.{h,cc}: multi-hop node-classification sampler over a host CSC graph with a
    GPU-cached sub-CSR (local / peer GPUs) for `cache_nids`."""

    def __init__(self, indptr, indices, probs, cache_nids, device_id):
        for t, name in ((indptr, "indptr"), (indices, "indices"), (probs, "probs")):
            check_cpu(t, name)
        self._id_dtype = indices.dtype
        self._cpu = (indptr, indices, probs)
        ip = _host_i64(indptr, "indptr")
        ix = _host_i64(indices, "indices")
        self._keep = [ip, ix]
        self.bias = probs.numel() > 0
        pr = None
        if self.bias:
            if probs.dtype != torch.float32:
                raise RuntimeError("probs must be float32")
            pr = probs.contiguous()
            self._keep.append(pr)
        cn = cache_nids.to(torch.int64).contiguous()
        self._keep.append(cn)
        # the reference's cache map holds ids of the cache list's type (hashmap.cu:18-31)
        self._cache_dtype = cache_nids.dtype if cache_nids.dtype in (torch.int32, torch.int64) \
            else torch.int64
        self.num_nodes = ip.numel() - 1
        h = c_vp()
        # pageable host arrays are copied by the library (never registered in place); pinned
        # ones (pin_memory(), _CAPI_tensor_pin_memory) are read in place
        check(lib.dgs_sampler_create(ptr(ip), ptr(ix), ptr(pr), self.num_nodes, ix.numel(),
                                     ptr(cn), cn.numel(), int(device_id), ctypes.byref(h)))
        self._h = h
        self._plans = {}
        self.device = torch.device("cuda", torch.cuda.current_device())

    def _CAPI_sample_node_classifiction(self, seeds, fan_out, replace=False):
        """sampler.cc:146-166 -> [(seeds, frontier, coo_row, coo_col)] per hop
        (hop h samples fan_out[L-1-h]); coo ids are local to (frontier, seeds).  Runs on the
        current stream; calls on different streams run concurrently."""
        return self._sample(seeds, fan_out, replace, None)

    def _sample_seeded(self, seeds, fan_out, replace, launch_seeds):
        """ADDITIVE: the same call with caller-drawn per-hop launch seeds (hop h uses
        launch_seeds[h]; draw them with dgs.ops.draw_launch_seeds)."""
        return self._sample_begin(seeds, fan_out, replace, launch_seeds).result()

    def _sample_begin(self, seeds, fan_out, replace=False, launch_seeds=None, host_async=False):
        """ADDITIVE: enqueue the whole call on the current stream and return at once; the
        returned handle's result() waits for the sizes and gives the call's blocks.  One call
        per stream may be outstanding (DistGNN.dataloading.PrefetchLoader keeps one per
        stream on several streams).  host_async: a library thread issues the launches, so
        this returns before they are enqueued -- nothing else may be enqueued on the stream
        until result()."""
        if launch_seeds is not None and len(launch_seeds) != len(fan_out):
            raise RuntimeError("launch_seeds needs one seed per hop")
        prep = self._prepare(seeds, fan_out)
        return self._begin_prepared(seeds, prep, replace, launch_seeds, host_async,
                                    stream_ptr(prep[0].device))

    def _begin_prepared(self, seeds, prep, replace, launch_seeds, host_async, stream,
                        wait_for=None, wait_event=None):
        """Enqueues a call whose int64 seeds and output buffer _prepare made, on `stream`
        (a c_void_p or int HIP stream), in one C-ABI call with the batch stream's wait:
        `wait_for` (an int HIP stream, 0 = the null stream) makes `stream` wait for the work
        enqueued on it so far; `wait_event` (an int hipEvent_t) makes it wait on that event."""
        s, L, fo, caps, total, buf, ptrs = prep
        st = stream if isinstance(stream, c_vp) else c_vp(stream)
        ls = None
        if L and launch_seeds is not None:
            ls = (ctypes.c_uint64 * L)(*[int(x) & 0xFFFFFFFFFFFFFFFF for x in launch_seeds])
        if L and wait_event is not None:
            check(lib.dgs_sampler_sample_begin_after(self._h, wait_event, s.data_ptr(),
                                                     s.numel(), fo, L, int(bool(replace)),
                                                     buf.data_ptr(), ls,
                                                     _SAMPLE_WAIT_EVENT | (1 if host_async else 0),
                                                     st))
        elif L and wait_for is not None:
            # the wait is requested by the flag: wait_for may be 0, the null stream
            check(lib.dgs_sampler_sample_begin_after(self._h, wait_for, s.data_ptr(),
                                                     s.numel(), fo, L, int(bool(replace)),
                                                     buf.data_ptr(), ls,
                                                     _SAMPLE_WAIT | (1 if host_async else 0),
                                                     st))
        elif L:
            check(lib.dgs_sampler_sample_begin(self._h, c_vp(s.data_ptr()), s.numel(), fo, L,
                                               int(bool(replace)), *ptrs, ls,
                                               1 if host_async else 0, st))
        elif wait_event is not None:
            check(lib.dgs_stream_wait_event(c_vp(wait_event), st))
        elif wait_for is not None:
            check(lib.dgs_stream_wait(c_vp(wait_for), st))
        return _PendingSample(self, seeds, s, L, caps, total, buf, st)

    def _sample(self, seeds, fan_out, replace, launch_seeds):
        """The synchronous call: every hop enqueued at once, then each hop's views are built as
        soon as its compaction publishes (U, nnz) -- while the later hops still run on the GPU
        (round 6: the views no longer wait for the whole call)."""
        if launch_seeds is not None:
            return self._sample_seeded(seeds, fan_out, replace, launch_seeds)
        s, L, fo, caps, total, buf, _ = self._prepare(seeds, fan_out, packed=True)
        if L == 0:
            return []
        st = stream_ptr(s.device)
        h_ = self._h
        check(lib.dgs_sampler_sample_packed_begin(h_, s.data_ptr(), s.numel(), fo, L,
                                                  int(bool(replace)), buf.data_ptr(), st))
        cast = self._id_dtype != torch.int64
        out, cur, off = [], seeds, 0
        un = (c_i64 * 2)()
        try:
            for h in range(L - 1):
                check(lib.dgs_sampler_sample_wait_hop(h_, L, h, un, st))
                f, e = caps[h]
                U, nnz = un[0], un[1]
                fr, r, c = (buf[off:off + U], buf[off + f:off + f + nnz],
                            buf[off + f + e:off + f + e + nnz])
                if cast:
                    fr, r, c = fr.to(self._id_dtype), r.to(self._id_dtype), c.to(self._id_dtype)
                out.append((cur, fr, r, c))
                cur, off = fr, off + f + 2 * e
        except BaseException:
            sizes = (c_i64 * (3 * L))()
            lib.dgs_sampler_sample_end(h_, L, sizes, st)  # ends the call (its error, if any,
            raise                                         # is the one raised here)
        sizes = (c_i64 * (3 * L))()
        check(lib.dgs_sampler_sample_end(h_, L, sizes, st))
        f, e = caps[L - 1]
        U, nnz = sizes[3 * L - 2], sizes[3 * L - 1]
        fr, r, c = buf[off:off + U], buf[off + f:off + f + nnz], buf[off + f + e:off + f + e + nnz]
        if cast:
            fr, r, c = fr.to(self._id_dtype), r.to(self._id_dtype), c.to(self._id_dtype)
        out.append((cur, fr, r, c))
        return out

    def _prepare(self, seeds, fan_out, packed=False, alloc_stream=None):
        """packed: no per-hop pointer arrays (the buffer goes to the C ABI whole).
        alloc_stream: the (stream_id, device_index, device_type) of the torch stream whose pool
        the output buffer comes from (the stream the call writes it on; default the current
        stream)."""
        check_cuda(seeds, "seeds")
        s = seeds if seeds.dtype == torch.int64 and seeds.is_contiguous() else \
            as_i64(seeds, "seeds")
        L = len(fan_out)
        if L == 0:
            return s, 0, None, [], 0, None, None
        key = (tuple(fan_out), s.numel())
        plan = self._plans.get(key)
        if plan is None:
            fo = i64_array(fan_out)
            fcap, ecap = (c_i64 * L)(), (c_i64 * L)()
            check(lib.dgs_sampler_bounds(self._h, s.numel(), fo, L, fcap, ecap))
            caps = [(int(fcap[h]), int(ecap[h])) for h in range(L)]
            plan = (fo, caps, sum(f + 2 * e for f, e in caps))
            self._plans[key] = plan
        fo, caps, total = plan
        # one allocation for every hop's (frontier, row, col) buffers
        if alloc_stream is None:
            buf = torch.empty(max(total, 1), dtype=torch.int64, device=s.device)
        elif _set_stream is None or _get_stream is None:  # no bare stream switch in this build
            with torch.cuda.stream(torch.cuda.Stream(stream_id=alloc_stream[0],
                                                     device_index=alloc_stream[1],
                                                     device_type=alloc_stream[2])):
                buf = torch.empty(max(total, 1), dtype=torch.int64, device=s.device)
        else:
            # a bare current-stream switch around the allocation (the stream context manager
            # costs several us of host time per batch, which a host-bound loader feels)
            cur = _get_stream(s.device.index)
            _set_stream(stream_id=alloc_stream[0], device_index=alloc_stream[1],
                        device_type=alloc_stream[2])
            try:
                buf = torch.empty(max(total, 1), dtype=torch.int64, device=s.device)
            finally:
                _set_stream(stream_id=cur[0], device_index=cur[1], device_type=cur[2])
        return s, L, fo, caps, total, buf, None if packed else plan_ptrs(buf.data_ptr(), caps)

    def _views(self, seeds, buf, caps, total, sizes, L, cast=True):
        # per hop [frontier f | rows e | cols e]: the three live prefixes and the pads after
        # them, as ONE split (round 4: one split_with_sizes into 6L pieces costs the host about
        # 2/3 of 3L separate slices, each of which is a full Python indexing call)
        parts = []
        for h in range(L):
            f, e = caps[h]
            U, nnz = sizes[3 * h + 1], sizes[3 * h + 2]
            parts += (U, f - U, nnz, e - nnz, nnz, e - nnz)
        rest = buf.numel() - total
        if rest:
            parts.append(rest)
        pieces = torch.split_with_sizes(buf, parts)
        out = []
        cur = seeds
        cast = cast and self._id_dtype != torch.int64
        for h in range(L):
            fr, r, c = pieces[6 * h], pieces[6 * h + 2], pieces[6 * h + 4]
            if cast:
                fr, r, c = fr.to(self._id_dtype), r.to(self._id_dtype), c.to(self._id_dtype)
            out.append((cur, fr, r, c))
            cur = fr
        return out

    def _num_contexts(self):
        """ADDITIVE (diagnostics): sampling contexts held, one per stream that sampled recently
        (at most DGS_SAMPLER_MAX_CTX, default 8)."""
        n = c_i64()
        check(lib.dgs_sampler_context_count(self._h, ctypes.byref(n)))
        return n.value

    def _CAPI_get_cpu_structure_tensors(self):
        indptr, indices, probs = self._cpu
        return indptr, indices, (probs if self.bias else None)

    def _CAPI_get_local_cache_structure_tensors(self):
        """Non-owning device views of this rank's cached sub-CSR (sampler.cc:183-195)."""
        pi, pe, pp = c_vp(), c_vp(), c_vp()
        nr, ne = c_i64(), c_i64()
        check(lib.dgs_sampler_local_cache(self._h, ctypes.byref(pi), ctypes.byref(nr),
                                          ctypes.byref(pe), ctypes.byref(ne), ctypes.byref(pp)))
        sub_indptr = device_view(pi.value, (nr.value + 1,), torch.int64, self)
        sub_indices = device_view(pe.value, (ne.value,), torch.int64, self)
        sub_probs = device_view(pp.value, (ne.value,), torch.float32, self) if self.bias else None
        return sub_indptr, sub_indices, sub_probs

    def _CAPI_get_local_cache_hashmap_tensors(self):
        """sampler.cc:197-201 -> (key, idx, devid): the reference's open-addressing cache map
        (hashmap.cu:15-77) -- 2 * _UpPower(total cached) slots of the cache lists' id type, -1
        where empty, every rank's list inserted with the reference's Murmur3 hash and probe
        sequence in its rotation order (local list last).  Built on the device when called."""
        n = c_i64()
        check(lib.dgs_sampler_cache_hashmap_capacity(self._h, ctypes.byref(n)))
        dt = self._cache_dtype
        key = torch.empty(n.value, dtype=dt, device=self.device)
        idx = torch.empty(n.value, dtype=dt, device=self.device)
        devid = torch.empty(n.value, dtype=dt, device=self.device)
        check(lib.dgs_sampler_cache_hashmap_fill(self._h, key.element_size(), ptr(key), ptr(idx),
                                                 ptr(devid), stream_ptr(self.device)))
        return key, idx, devid

    def _local_cache_map_compact(self):
        """ADDITIVE: (key, idx, devid) with one entry per cached node, in node-id order, local
        entries taking priority (the lookup results of the map above, int64)."""
        n = c_i64()
        check(lib.dgs_sampler_cache_map_size(self._h, ctypes.byref(n)))
        key = torch.empty(n.value, dtype=torch.int64, device=self.device)
        idx = torch.empty(n.value, dtype=torch.int64, device=self.device)
        devid = torch.empty(n.value, dtype=torch.int64, device=self.device)
        check(lib.dgs_sampler_cache_map_fill(self._h, ptr(key), ptr(idx), ptr(devid),
                                             stream_ptr(self.device)))
        return key, idx, devid

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.dgs_sampler_destroy(h)
            self._h = None


class P2PCacheFeatureServer:
    """feature_server.cc: host feature matrix with a per-GPU HBM cache of `cache_nids`
    rows, pooled across GPUs (peer rows are read one-sided over xGMI)."""

    def __init__(self, data, cache_nids, device_id):
        check_cpu(data, "data")
        if data.dim() == 0:
            raise RuntimeError("data must have at least one dimension")
        self._cpu = data
        d = data.contiguous()
        self._keep = [d]
        self._stride, self._row_bytes = row_bytes(d)
        self._dtype = d.dtype
        self._shape_tail = tuple(d.shape[1:])
        cn = cache_nids.to(torch.int64).contiguous()
        self._keep.append(cn)
        h = c_vp()
        check(lib.dgs_feature_server_create(ptr(d), d.shape[0], self._row_bytes, ptr(cn),
                                            cn.numel(), int(device_id), ctypes.byref(h)))
        self._h = h
        self.device = torch.device("cuda", torch.cuda.current_device())

    def _CAPI_get_cpu_feature(self):
        return self._cpu

    def _CAPI_get_gpu_feature(self):
        p, n = c_vp(), c_i64()
        check(lib.dgs_feature_server_local_cache(self._h, ctypes.byref(p), ctypes.byref(n)))
        if not p.value:
            return None
        return device_view(p.value, (n.value,) + self._shape_tail, self._dtype, self)

    def _CAPI_get_feature(self, nids):
        """feature_server.cc:69-74 -> [n, stride] (2-D, feature_ops.cu:110-112)."""
        check_cuda(nids, "nids")
        n = nids if nids.dtype == torch.int64 and nids.is_contiguous() else as_i64(nids, "nids")
        out = torch.empty((n.numel(), self._stride), dtype=self._dtype, device=n.device)
        check(lib.dgs_feature_server_gather(self._h, c_vp(n.data_ptr()), n.numel(),
                                            c_vp(out.data_ptr()), stream_ptr(n.device)))
        return out

    def _get_feature_alloc(self, nids):
        """Loader fast path, part 1: the output of _get_feature_into (current stream).  Its
        room is rounded up to 1/8 steps between powers of two (a view of the first rows is
        returned): batches whose row counts differ a little then reuse one cached block, where
        a batch slightly larger than any before would make the caching allocator map a new
        segment inside the loop (round 5: the one hipMalloc left in the bench's timed region)."""
        n = nids.numel()
        room = n
        if n > 4096:
            step = (1 << (n.bit_length() - 1)) >> 3
            room = (n + step - 1) // step * step
        out = torch.empty((room, self._stride), dtype=self._dtype, device=nids.device)
        return out[:n] if room != n else out

    def _get_feature_into(self, nids, out, stream):
        """Loader fast path, part 2: gather of int64 contiguous device `nids` into `out` on HIP
        stream `stream` (int)."""
        check(lib.dgs_feature_server_gather(self._h, c_vp(nids.data_ptr()), nids.numel(),
                                            c_vp(out.data_ptr()), c_vp(stream)))

    def _layout(self):
        """ADDITIVE: -1 = address-table gather, w >= 0 = strided layout over 2^w GPUs."""
        w = ctypes.c_int()
        check(lib.dgs_feature_server_layout(self._h, ctypes.byref(w)))
        return w.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.dgs_feature_server_destroy(h)
            self._h = None


_SAMPLE_WAIT = 2  # DGS_SAMPLE_WAIT (include/dgs_amd.h)
_SAMPLE_WAIT_EVENT = 4  # DGS_SAMPLE_WAIT_EVENT
_get_stream = getattr(torch._C, "_cuda_getCurrentStream", None)
_set_stream = getattr(torch._C, "_cuda_setStream", None)


class _PendingSample:
    """A sample call enqueued by P2PCacheSampler._sample_begin; result() (once) waits for the
    sizes its last kernel publishes and returns the per-hop (seeds, frontier, row, col)."""

    def __init__(self, owner, seeds, s64, L, caps, total, buf, stream):
        self._owner, self._seeds, self._s64 = owner, seeds, s64
        self._L, self._caps, self._total, self._buf, self._stream = L, caps, total, buf, stream
        self._out = None

    @property
    def buffer(self):
        """The call's output buffer until result() has built the views (then None)."""
        return self._buf

    def result(self, cast=True):
        """cast=False leaves int32-id graphs' blocks as int64 (the caller casts them once its
        stream is ordered after the call's)."""
        if self._out is None:
            if self._L == 0:
                self._out = []
            else:
                if self._owner._h is None:  # destroyed (e.g. finalised first in a GC cycle)
                    raise RuntimeError("dgs: the sampler of this call has been destroyed")
                sizes = (c_i64 * (3 * self._L))()
                check(lib.dgs_sampler_sample_end(self._owner._h, self._L, sizes, self._stream))
                self._out = self._owner._views(self._seeds, self._buf, self._caps, self._total,
                                               sizes, self._L, cast)
            self._s64 = self._buf = None
        return self._out
