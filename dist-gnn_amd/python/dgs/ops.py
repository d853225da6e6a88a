"""dgs.ops -- mirror of the reference's `m_ops` submodule (src/pybind.cc:47-77).

Every function keeps the reference name, argument order, dtype rules and return shape; the
work is done by libdgs_amd.so (HIP kernels on the current device, current stream).
"""
import ctypes

import torch

from . import _lib
from ._lib import c_i64, check, i64_array, lib, stream_ptr, vp_array
from ._util import as_i64, check_cuda, ptr, row_bytes

__all__ = [
    "_CAPI_get_unique_id", "_CAPI_set_nccl", "_CAPI_compute_frontier_heat",
    "_CAPI_compute_frontier_heat_with_bias", "_CAPI_tensor_pin_memory",
    "_CAPI_tensor_unpin_memory", "_CAPI_cuda_sample_neighbors",
    "_CAPI_cuda_sample_neighbors_bias", "_CAPI_cuda_sampled_tensor_relabel",
    "_CAPI_cuda_index_select", "_Test_Randn", "_Test_NCCLTensorAllGather",
    "_Test_GetLocalRank", "_Test_GetWorldSize", "_Test_ExtractEdgeData", "_Test_ExtractIndptr",
    "_CAPI_set_random_seed", "_CAPI_set_host_comm", "draw_launch_seeds", "_Test_BiasKeyBounds",
]

# host storage registered by _CAPI_tensor_pin_memory: data_ptr -> (the tensor, the registered
# storage base).  Holding the tensor keeps its memory alive while registered (a registration
# outliving its allocation would make HIP reject later copies through memory the allocator
# reuses).
_registered = {}


def _cuda_dev():
    return torch.device("cuda", torch.cuda.current_device())


# ------------------------------------------------------------------ communicator
def _CAPI_get_unique_id():
    """nccl_context.cc:13-18 -- RCCL unique id packed into 16 int64."""
    out = (c_i64 * 16)()
    check(lib.dgs_get_unique_id(out))
    return [int(x) for x in out]


def _CAPI_set_nccl(nranks, unique_id_array, rank):
    """nccl_context.cc:20-45."""
    ids = i64_array(unique_id_array)
    check(lib.dgs_set_nccl(int(nranks), ids, len(unique_id_array), int(rank)))


_HOST_AG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                            ctypes.c_void_p)
_HOST_BAR = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
_host_comm_refs = []


def _CAPI_set_host_comm(group=None):
    """ADDITIVE: run the library's setup collectives (IPC-handle / cache-list all-gathers,
    barriers) over an existing torch.distributed group (e.g. gloo) instead of RCCL.  Used by the
    multi-rank tests, where several ranks share one GPU; the hot path is unchanged."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)

    def allgather(send, nbytes, recv, _ctx):
        try:
            src = torch.empty(nbytes, dtype=torch.uint8)
            ctypes.memmove(src.data_ptr(), send, nbytes)
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(outs, src, group=group)
            for i, o in enumerate(outs):
                ctypes.memmove(recv + i * nbytes, o.data_ptr(), nbytes)
            return 0
        except Exception:  # pragma: no cover - surfaced as a library error
            return 1

    def barrier(_ctx):
        try:
            dist.barrier(group)
            return 0
        except Exception:  # pragma: no cover
            return 1

    ag, bar = _HOST_AG(allgather), _HOST_BAR(barrier)
    _host_comm_refs.extend([ag, bar])
    check(lib.dgs_set_host_comm(world, rank, ctypes.cast(ag, ctypes.c_void_p),
                                ctypes.cast(bar, ctypes.c_void_p), None))


def _Test_GetLocalRank():
    return int(lib.dgs_get_local_rank())


def _Test_GetWorldSize():
    return int(lib.dgs_get_world_size())


def _Test_Randn():
    """context/context.h:22-27 -- next launch seed (uint64)."""
    return int(lib.dgs_randn_uint64())


def draw_launch_seeds(n):
    """ADDITIVE: the next n launch seeds of the global engine, drawn under one lock (what one
    n-hop sample call would draw), for P2PCacheSampler._sample_seeded."""
    out = (ctypes.c_uint64 * int(n))()
    check(lib.dgs_randn_uint64_n(int(n), out))
    return [int(x) for x in out]


def _CAPI_set_random_seed(seed):
    """ADDITIVE: reseed the launch-seed engine (std::mt19937_64) for reproducible sampling."""
    check(lib.dgs_set_random_seed(int(seed) & 0xFFFFFFFFFFFFFFFF))


def _Test_NCCLTensorAllGather(local_tensor):
    """nccl_context.cc:52-112 -- sizes, then payload via grouped send/recv."""
    check_cuda(local_tensor, "local_tensor")
    t = local_tensor.contiguous()
    world = _Test_GetWorldSize()
    rank = _Test_GetLocalRank()
    sizes = (c_i64 * world)()
    check(lib.dgs_allgather_sizes(t.numel(), sizes))
    out = [t if i == rank else torch.empty(int(sizes[i]), dtype=t.dtype, device=t.device)
           for i in range(world)]
    nbytes = i64_array([int(sizes[i]) * t.element_size() for i in range(world)])
    check(lib.dgs_allgather_bytes(ptr(t), t.numel() * t.element_size(),
                                  vp_array([o.data_ptr() for o in out]), nbytes, stream_ptr()))
    return out


# ------------------------------------------------------------------ pinning
def _CAPI_tensor_pin_memory(data):
    """pin_memory.cc:7-12 -- register the tensor's host storage (mapped) in place.  The whole
    storage is registered (the reference registers the tensor's own range): any view of the
    buffer, including a later service's, then maps through this one registration."""
    if data.is_cuda or data.is_pinned() or data.numel() == 0:
        return
    p = data.data_ptr()
    if p in _registered:
        return
    st = data.untyped_storage()
    check(lib.dgs_host_register(ctypes.c_void_p(st.data_ptr()), st.nbytes()))
    _registered[p] = (data, st.data_ptr())


def _CAPI_tensor_unpin_memory(data):
    """pin_memory.cc:14-19.  The reference early-returns when is_pinned() (so it never
    unregisters); here storage registered by _CAPI_tensor_pin_memory is released."""
    if data.is_cuda:
        return
    p = data.data_ptr()
    if p in _registered:
        check(lib.dgs_host_unregister(ctypes.c_void_p(_registered[p][1])))
        del _registered[p]


# ------------------------------------------------------------------ sampling
def _sample(seeds, indptr, indices, probs, num_picks, replace):
    check_cuda(seeds, "seeds")
    if seeds.dtype != indices.dtype:
        raise RuntimeError("seeds dtype must equal indices dtype")
    out_dtype = indices.dtype
    s, ip, ix = as_i64(seeds, "seeds"), as_i64(indptr, "indptr"), as_i64(indices, "indices")
    pr = None
    if probs is not None:
        if probs.dtype != torch.float32:
            raise RuntimeError("probs must be float32")
        pr = probs.contiguous()
    cap = s.numel() * int(num_picks)
    dev = seeds.device
    row = torch.empty(max(cap, 0), dtype=torch.int64, device=dev)
    col = torch.empty(max(cap, 0), dtype=torch.int64, device=dev)
    nnz = c_i64(0)
    check(lib.dgs_sample_neighbors(ptr(s), s.numel(), ptr(ip), ptr(ix), ptr(pr), int(num_picks),
                                   int(bool(replace)), ptr(row), ptr(col), ctypes.byref(nnz),
                                   stream_ptr(dev)))
    row, col = row[:nnz.value], col[:nnz.value]
    if out_dtype != torch.int64:
        row, col = row.to(out_dtype), col.to(out_dtype)
    return row, col


def _CAPI_cuda_sample_neighbors(seeds, indptr, indices, num_picks, replace):
    """rowwise_sampling.cu:143-189 -> (coo_row, coo_col)."""
    return _sample(seeds, indptr, indices, None, num_picks, replace)


def _CAPI_cuda_sample_neighbors_bias(seeds, indptr, indices, probs, num_picks, replace):
    """rowwise_sampling_bias.cu:226-288 -> (coo_row, coo_col)."""
    return _sample(seeds, indptr, indices, probs, num_picks, replace)


def _CAPI_cuda_sampled_tensor_relabel(mapping_tensors, requiring_relabel_tensors):
    """tensor_relabel.cu:182-205 -> (unique, [relabeled tensors])."""
    maps = [as_i64(t, "mapping tensor") for t in mapping_tensors]
    reqs = [as_i64(t, "relabel tensor") for t in requiring_relabel_tensors]
    dtype = requiring_relabel_tensors[0].dtype if requiring_relabel_tensors else torch.int64
    dev = maps[0].device if maps else _cuda_dev()
    nm = sum(t.numel() for t in maps)
    uniq = torch.empty(nm, dtype=torch.int64, device=dev)
    outs = [torch.empty(t.numel(), dtype=torch.int64, device=dev) for t in reqs]
    nu = c_i64(0)
    check(lib.dgs_relabel(vp_array([t.data_ptr() for t in maps]),
                          i64_array([t.numel() for t in maps]), len(maps),
                          vp_array([t.data_ptr() for t in reqs]),
                          i64_array([t.numel() for t in reqs]), len(reqs), ptr(uniq),
                          ctypes.byref(nu), vp_array([o.data_ptr() for o in outs]),
                          stream_ptr(dev)))
    uniq = uniq[:nu.value]
    if dtype != torch.int64:
        uniq = uniq.to(dtype)
        outs = [o.to(dtype) for o in outs]
    outs = [o.view(r.shape) for o, r in zip(outs, requiring_relabel_tensors)]
    return uniq, outs


# ------------------------------------------------------------------ gather
def _CAPI_cuda_index_select(data, nid):
    """feature_ops.cu:173-210 -- out = data[nid] on the current CUDA device, keeping the
    trailing shape; data may be a CUDA tensor or pinned host memory."""
    if nid.dtype not in (torch.int32, torch.int64):
        raise RuntimeError("ID can only be int32 or int64")
    if data.dtype not in (torch.int32, torch.int64, torch.float32):
        raise RuntimeError("Value can only be int32 or int64 or float32")
    d = data.contiguous()
    n = nid.contiguous()
    _, rb = row_bytes(d)
    dev = n.device if n.is_cuda else _cuda_dev()
    out = torch.empty((n.numel(),) + tuple(d.shape[1:]), dtype=d.dtype, device=dev)
    rows = d.shape[0] if d.dim() > 0 else 1
    check(lib.dgs_index_select(ptr(d), rows, rb, ptr(n), n.element_size(), n.numel(), ptr(out),
                               stream_ptr(dev)))
    return out


def _index_select_into(data, nid, out, stream):
    """Loader fast path: out = data[nid] for contiguous device tensors `data`
    (int32/int64/float32), int64 `nid` and `out`, on HIP stream `stream` (int)."""
    rb = data.element_size()
    for d in data.shape[1:]:
        rb *= int(d)
    check(lib.dgs_index_select_device(ctypes.c_void_p(data.data_ptr()), data.shape[0], rb,
                                      ctypes.c_void_p(nid.data_ptr()), 8, nid.numel(),
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))


def _loader_gather(sampler, server, producer, consumer, nids, x, labels, label_row_bytes, seeds,
                   y):
    """ADDITIVE (PrefetchLoader): `consumer` waits for `producer` (the sample call of
    `sampler` just ended on it; sampler None: any work), then x = features[nids] (server may be
    None) and y = labels[seeds] (labels may be None), on `consumer`; one C-ABI call.  All
    tensors contiguous device tensors, nids and seeds int64; streams are ints."""
    check(lib.dgs_loader_gather(
        sampler._h if sampler is not None else None,
        server._h if server is not None else None, producer, consumer,
        nids.data_ptr() if nids is not None else None, nids.numel() if nids is not None else 0,
        x.data_ptr() if x is not None else None,
        labels.data_ptr() if labels is not None else None,
        labels.shape[0] if labels is not None else 0, label_row_bytes,
        seeds.data_ptr(), seeds.numel() if labels is not None else 0,
        y.data_ptr() if y is not None else None))


def _check_async_errors():
    """ADDITIVE: raises RuntimeError if a gather kernel of this process met an id outside its
    source's rows since the last check (the kernel read row 0 instead; the reference reads out
    of bounds).  Every gather entry point checks this first, so such an error surfaces at the
    next gather at the latest.  No synchronisation: synchronise first to see queued work's."""
    check(lib.dgs_check_async_errors())


def _last_gather_tag():
    """ADDITIVE: the call tag ("gather call #") of this thread's last gather launch."""
    t = ctypes.c_uint64()
    check(lib.dgs_last_gather_tag(ctypes.byref(t)))
    return t.value


def _host_registrations():
    """ADDITIVE (diagnostics, tests): the library's live host registrations as a list of
    dicts {base, bytes, refs, pins}.  Only _CAPI_tensor_pin_memory registers caller memory;
    services copy pageable arrays instead."""
    n = c_i64()
    check(lib.dgs_host_registrations(0, None, None, None, None, ctypes.byref(n)))
    k = n.value
    if k == 0:
        return []
    bases, nb = (ctypes.c_uint64 * k)(), (c_i64 * k)()
    refs, pins = (c_i64 * k)(), (c_i64 * k)()
    check(lib.dgs_host_registrations(k, bases, nb, refs, pins, ctypes.byref(n)))
    return [{"base": int(bases[i]), "bytes": int(nb[i]), "refs": int(refs[i]),
             "pins": int(pins[i])} for i in range(min(k, n.value))]


def _host_memory_state():
    """ADDITIVE (diagnostics, tests): {registrations, mirror_bytes, mirrors} -- live
    registrations and the library's pinned host mirrors (services with host-resident rows)."""
    r, b, m = c_i64(), c_i64(), c_i64()
    check(lib.dgs_host_memory_state(ctypes.byref(r), ctypes.byref(b), ctypes.byref(m)))
    return {"registrations": r.value, "mirror_bytes": b.value, "mirrors": m.value}


def _stream_create(priority=0):
    """ADDITIVE: a new non-blocking HIP stream (int handle) owned by the caller; hand it to
    torch with torch.cuda.ExternalStream.  Unlike torch's pooled streams it is never given to
    anyone else."""
    out = ctypes.c_void_p()
    check(lib.dgs_stream_create(int(priority), ctypes.byref(out)))
    return out.value


def _stream_wait(producer, consumer):
    """ADDITIVE: HIP stream `consumer` waits for the work enqueued on `producer` so far (ints)."""
    check(lib.dgs_stream_wait(ctypes.c_void_p(producer), ctypes.c_void_p(consumer)))


# ------------------------------------------------------------------ cache helpers
def _Test_ExtractIndptr(nids, indptr):
    """utils.cu:12-42."""
    n = as_i64(nids, "nids")
    ip = as_i64(indptr, "indptr")
    dev = n.device if n.is_cuda else _cuda_dev()
    out = torch.empty(n.numel() + 1, dtype=torch.int64, device=dev)
    check(lib.dgs_extract_indptr(ptr(n), n.numel(), ptr(ip), ptr(out), stream_ptr(dev)))
    return out.to(indptr.dtype) if indptr.dtype != torch.int64 else out


def _Test_ExtractEdgeData(nids, indptr, sub_indptr, edge_data):
    """utils.cu:44-101."""
    n = as_i64(nids, "nids")
    ip = as_i64(indptr, "indptr")
    sp = as_i64(sub_indptr, "sub_indptr")
    ed = edge_data.contiguous()
    total = int(sp[-1].item()) if sp.numel() else 0
    dev = n.device if n.is_cuda else _cuda_dev()
    out = torch.empty(total, dtype=ed.dtype, device=dev)
    check(lib.dgs_extract_edge_data(ptr(n), n.numel(), ptr(ip), ptr(sp), ptr(ed),
                                    ed.element_size(), ptr(out), stream_ptr(dev)))
    return out


def _Test_BiasKeyBounds(x, p, thr):
    """ADDITIVE test op (include/dgs_amd.h dgs_test_bias_bounds): for 32-bit draws x (int64
    values in [0, 2^32)), probabilities p and thresholds thr (float32, CUDA, equal sizes) ->
    (exact A-Res key, its lower bound, reject flags: bit 0 streamed-hub filter, bit 1 row
    filter, each set only when the key is certainly below thr)."""
    for t, name in ((x, "x"), (p, "p"), (thr, "thr")):
        check_cuda(t, name)
    if not (x.numel() == p.numel() == thr.numel()):
        raise RuntimeError("x, p and thr need equal sizes")
    if p.dtype != torch.float32 or thr.dtype != torch.float32:
        raise RuntimeError("p and thr must be float32")
    xi = x.to(torch.int64)
    x32 = torch.where(xi >= 2 ** 31, xi - 2 ** 32, xi).to(torch.int32).contiguous()
    pc, tc = p.contiguous(), thr.contiguous()
    key = torch.empty_like(pc)
    low = torch.empty_like(pc)
    flags = torch.empty(pc.numel(), dtype=torch.uint8, device=pc.device)
    check(lib.dgs_test_bias_bounds(ptr(x32), ptr(pc), ptr(tc), pc.numel(), ptr(key), ptr(low),
                                   ptr(flags), stream_ptr(pc.device)))
    return key, low, flags


# ------------------------------------------------------------------ heat
def _heat(seeds, indptr, indices, probs, seeds_heat, num_picks, indptr_diff, deterministic):
    s, ip, ix = as_i64(seeds, "seeds"), as_i64(indptr, "indptr"), as_i64(indices, "indices")
    if seeds_heat.dtype != torch.float32:
        raise RuntimeError("heat must be float32")
    fh = torch.zeros_like(seeds_heat)
    pr = probs.contiguous() if probs is not None else None
    fn = lib.dgs_compute_frontier_heat_fixed if deterministic else lib.dgs_compute_frontier_heat
    check(fn(ptr(s), s.numel(), ptr(ip), ptr(ix), ptr(pr), ptr(seeds_heat), seeds_heat.numel(),
             int(num_picks), int(indptr_diff), ptr(fh), stream_ptr(fh.device)))
    return fh


def _CAPI_compute_frontier_heat(seeds, indptr, indices, seeds_heat, num_picks, indptr_diff,
                                deterministic=False):
    """preprocess_heat.cu:35-56.  ADDITIVE deterministic=True: fixed-point accumulation
    (order-independent; see dgs_compute_frontier_heat_fixed)."""
    return _heat(seeds, indptr, indices, None, seeds_heat, num_picks, indptr_diff,
                 deterministic)


def _CAPI_compute_frontier_heat_with_bias(seeds, indptr, indices, probs, seeds_heat, num_picks,
                                          indptr_diff, deterministic=False):
    """preprocess_heat.cu:100-121 (processes seeds.numel() - 1 seeds, as the reference)."""
    return _heat(seeds, indptr, indices, probs, seeds_heat, num_picks, indptr_diff,
                 deterministic)


PROFILE_GATHER, PROFILE_SAMPLE, PROFILE_SELECT = 1, 2, 4


def profile_enable(on=True):
    """ADDITIVE instrumentation: True = everything, False = off, or a PROFILE_* bit mask."""
    mask = (7 if on else 0) if isinstance(on, bool) else int(on)
    check(lib.dgs_profile_enable(mask))


def profile_read():
    gm, gn, sm, sn = ctypes.c_double(), c_i64(), ctypes.c_double(), c_i64()
    xm, xn = ctypes.c_double(), c_i64()
    check(lib.dgs_profile_read(ctypes.byref(gm), ctypes.byref(gn), ctypes.byref(sm),
                               ctypes.byref(sn), ctypes.byref(xm), ctypes.byref(xn)))
    return {"gather_ms": gm.value, "gather_launches": gn.value, "sample_ms": sm.value,
            "sample_calls": sn.value, "select_ms": xm.value, "select_launches": xn.value}


_lib  # noqa: B018  (keep module import for side effects)
