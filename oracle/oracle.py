"""CPU oracle for the DGS sampling / relabel / gather path -- TEST INFRASTRUCTURE ONLY.

This module wraps oracle/build/liboracle.so (a plain-C restatement of the reference
algorithms, see dgs_oracle.h for the file:line each function follows).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import it, and only as the
checker; the product path (dist-gnn_amd/) never imports, links or calls it.

Parity status: pinned by the Philox / mt19937_64 known-answer vectors and the
hand-derived known answers of the reference's own tests (tests/golden/); beyond those
the reference (CUDA only, no golden outputs) could not be run here -- see DESIGN.md.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_f32p = ctypes.POINTER(ctypes.c_float)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_philox_draw.restype = ctypes.c_uint32
        L.oracle_philox_draw.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_mt64_next.restype = ctypes.c_uint64
        L.oracle_log2f.restype = ctypes.c_float
        L.oracle_log2f.argtypes = [ctypes.c_float]
        L.oracle_ares_key.restype = ctypes.c_float
        L.oracle_ares_key.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_curand.restype = ctypes.c_uint32
        L.oracle_curand_uniform.restype = ctypes.c_float
        L.oracle_curand_init.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p]
        for name in ("oracle_sample_uniform", "oracle_sample_bias", "oracle_relabel",
                     "oracle_sample_uniform_omp", "oracle_sample_bias_omp"):
            getattr(L, name).restype = ctypes.c_int64
        L.oracle_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t=_i64p):
    return a.ctypes.data_as(t)


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


# ---------------------------------------------------------------- RNG
def philox4x32_10(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox4x32_10(_p(c, _u32p), _p(k, _u32p), _p(out, _u32p))
    return out


def philox_draw(seed, subsequence, j):
    return lib().oracle_philox_draw(seed, subsequence, j)


class _PhiloxState(ctypes.Structure):
    _fields_ = [("ctr", ctypes.c_uint32 * 4), ("key", ctypes.c_uint32 * 2),
                ("output", ctypes.c_uint32 * 4), ("state", ctypes.c_uint32)]


def curand_stream(seed, subsequence, offset, n, uniform=False):
    st = _PhiloxState()
    L = lib()
    L.oracle_curand_init(seed, subsequence, offset, ctypes.byref(st))
    if uniform:
        return np.array([L.oracle_curand_uniform(ctypes.byref(st)) for _ in range(n)],
                        dtype=np.float32)
    return np.array([L.oracle_curand(ctypes.byref(st)) for _ in range(n)], dtype=np.uint32)


class MT64(ctypes.Structure):
    """std::mt19937_64 -- the reference's per-launch seed source (context/context.h:7-21)."""
    _fields_ = [("mt", ctypes.c_uint64 * 312), ("idx", ctypes.c_int)]

    def __init__(self, seed):
        super().__init__()
        lib().oracle_mt64_seed(ctypes.byref(self), ctypes.c_uint64(seed))

    def next(self):
        return lib().oracle_mt64_next(ctypes.byref(self))


def launch_seeds(seed, n):
    g = MT64(seed)
    return [g.next() for _ in range(n)]


def log2f(u):
    return lib().oracle_log2f(u)


def ares_key(u, p):
    return lib().oracle_ares_key(u, p)


def curand_uniform_of(x):
    """curand_uniform() of raw 32-bit draws x (uint32 array): RN(float(x) 2^-32 + 2^-33) -- the
    scaled float is exact, so one float64 sum rounded once to float32 reproduces the fma."""
    xf = np.asarray(x, dtype=np.uint64).astype(np.float32).astype(np.float64)
    return (xf * 2.0 ** -32 + 2.0 ** -33).astype(np.float32)


def ares_keys(u, p):
    """Vectorised ares_key (float32 arrays)."""
    u = np.ascontiguousarray(u, dtype=np.float32)
    p = np.ascontiguousarray(p, dtype=np.float32)
    out = np.empty_like(u)
    f = ctypes.POINTER(ctypes.c_float)
    lib().oracle_ares_keys(u.ctypes.data_as(f), p.ctypes.data_as(f), out.ctypes.data_as(f),
                           ctypes.c_int64(u.size))
    return out


# ---------------------------------------------------------------- sampling
def sample_uniform(seeds, indptr, indices, k, replace, launch_seed, nthreads=1):
    seeds, indptr, indices = _i64(seeds), _i64(indptr), _i64(indices)
    S = seeds.size
    cap = max(S * k, 1)
    row = np.empty(cap, np.int64)
    col = np.empty(cap, np.int64)
    if nthreads == 1:
        nnz = lib().oracle_sample_uniform(_p(seeds), S, _p(indptr), _p(indices), k,
                                          int(replace), ctypes.c_uint64(launch_seed),
                                          _p(row), _p(col))
    else:
        nnz = lib().oracle_sample_uniform_omp(_p(seeds), S, _p(indptr), _p(indices), k,
                                              int(replace), ctypes.c_uint64(launch_seed),
                                              _p(row), _p(col), nthreads)
    return row[:nnz].copy(), col[:nnz].copy()


def sample_bias(seeds, indptr, indices, probs, k, replace, launch_seed, nthreads=1):
    seeds, indptr, indices = _i64(seeds), _i64(indptr), _i64(indices)
    probs = np.ascontiguousarray(np.asarray(probs, dtype=np.float32))
    S = seeds.size
    cap = max(S * k, 1)
    row = np.empty(cap, np.int64)
    col = np.empty(cap, np.int64)
    nnz = lib().oracle_sample_bias_omp(_p(seeds), S, _p(indptr), _p(indices), _p(probs, _f32p),
                                       k, int(replace), ctypes.c_uint64(launch_seed), _p(row),
                                       _p(col), int(nthreads))
    return row[:nnz].copy(), col[:nnz].copy()


def relabel(mapping_list, requiring_list):
    """TensorRelabelCUDA semantics: (unique, [relabeled tensors split as the inputs])."""
    mapping = _i64(np.concatenate([np.asarray(m, np.int64) for m in mapping_list])
                   if mapping_list else np.zeros(0, np.int64))
    sizes = [np.asarray(r).size for r in requiring_list]
    req = _i64(np.concatenate([np.asarray(r, np.int64) for r in requiring_list])
               if requiring_list else np.zeros(0, np.int64))
    uniq = np.empty(max(mapping.size, 1), np.int64)
    rel = np.empty(max(req.size, 1), np.int64)
    u = lib().oracle_relabel(_p(mapping), mapping.size, _p(req), req.size, _p(uniq), _p(rel))
    out, off = [], 0
    for s in sizes:
        out.append(rel[off:off + s].copy())
        off += s
    return uniq[:u].copy(), out


def node_classification_sample(seeds, indptr, indices, fan_out, replace, launch_seeds_list,
                               probs=None):
    """P2PCacheSampler::NodeClassifictionSample semantics -> list of (seeds, frontier, row, col)."""
    seeds, indptr, indices = _i64(seeds), _i64(indptr), _i64(indices)
    L = len(fan_out)
    fo = _i64(fan_out)
    fcap = np.zeros(L, np.int64)
    ecap = np.zeros(L, np.int64)
    lib().oracle_nc_bounds(ctypes.c_int64(seeds.size), _p(fo), L, _p(fcap), _p(ecap))
    fronts = [np.empty(max(int(c), 1), np.int64) for c in fcap]
    rows = [np.empty(max(int(c), 1), np.int64) for c in ecap]
    cols = [np.empty(max(int(c), 1), np.int64) for c in ecap]
    arr_t = _i64p * L
    fptr = arr_t(*[_p(a) for a in fronts])
    rptr = arr_t(*[_p(a) for a in rows])
    cptr = arr_t(*[_p(a) for a in cols])
    ls = np.asarray(launch_seeds_list[:L], dtype=np.uint64)
    sizes = np.zeros(3 * L, np.int64)
    pp = None
    if probs is not None:
        probs = np.ascontiguousarray(np.asarray(probs, np.float32))
        pp = _p(probs, _f32p)
    lib().oracle_node_classification_sample(_p(seeds), ctypes.c_int64(seeds.size), _p(indptr),
                                            _p(indices), pp, _p(fo), L, int(replace),
                                            _p(ls, _u64p), fptr, rptr, cptr, _p(sizes))
    out = []
    cur = seeds
    for h in range(L):
        S, U, nnz = sizes[3 * h:3 * h + 3]
        fr = fronts[h][:U].copy()
        out.append((cur.copy(), fr, rows[h][:nnz].copy(), cols[h][:nnz].copy()))
        cur = fr
    return out


# ---------------------------------------------------------------- extract / gather / heat
def extract_indptr(nids, indptr):
    nids, indptr = _i64(nids), _i64(indptr)
    out = np.empty(nids.size + 1, np.int64)
    lib().oracle_extract_indptr(_p(nids), nids.size, _p(indptr), _p(out))
    return out


def extract_edge_data(nids, indptr, sub_indptr, edge_data):
    nids, indptr, sub_indptr = _i64(nids), _i64(indptr), _i64(sub_indptr)
    ed = np.ascontiguousarray(edge_data)
    out = np.empty(int(sub_indptr[-1]) if sub_indptr.size else 0, dtype=ed.dtype)
    lib().oracle_extract_edge_data(_p(nids), nids.size, _p(indptr), _p(sub_indptr),
                                   ed.ctypes.data_as(ctypes.c_void_p), ed.itemsize,
                                   out.ctypes.data_as(ctypes.c_void_p))
    return out


def index_select(data, nids, nthreads=1):
    data = np.ascontiguousarray(data)
    nids = _i64(nids)
    out = np.empty((nids.size,) + data.shape[1:], dtype=data.dtype)
    row_bytes = data.itemsize * (int(np.prod(data.shape[1:])) if data.ndim > 1 else 1)
    lib().oracle_index_select(data.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(row_bytes),
                              _p(nids), ctypes.c_int64(nids.size),
                              out.ctypes.data_as(ctypes.c_void_p), nthreads)
    return out


def frontier_heat(seeds, indptr, indices, seeds_heat, num_picks, indptr_diff=0, probs=None):
    seeds, indptr, indices = _i64(seeds), _i64(indptr), _i64(indices)
    sh = np.ascontiguousarray(np.asarray(seeds_heat, np.float32))
    out = np.empty(sh.size, np.float32)
    if probs is None:
        lib().oracle_frontier_heat(_p(seeds), ctypes.c_int64(seeds.size), _p(indptr),
                                   _p(indices), _p(sh, _f32p), ctypes.c_int64(num_picks),
                                   ctypes.c_int64(indptr_diff), ctypes.c_int64(sh.size),
                                   _p(out, _f32p))
    else:
        pr = np.ascontiguousarray(np.asarray(probs, np.float32))
        lib().oracle_frontier_heat_with_bias(_p(seeds), ctypes.c_int64(seeds.size), _p(indptr),
                                             _p(indices), _p(pr, _f32p), _p(sh, _f32p),
                                             ctypes.c_int64(num_picks),
                                             ctypes.c_int64(indptr_diff),
                                             ctypes.c_int64(sh.size), _p(out, _f32p))
    return out


def max_threads():
    return lib().oracle_max_threads()


# ------------------------------------------------------------------ the reference's cache map
_M32 = 0xFFFFFFFF
_M64 = 0xFFFFFFFFFFFFFFFF


def _murmur32(k):
    """hashmap.h:52-59 (Hash32Shift)."""
    k &= _M32
    k ^= k >> 16
    k = (k * 0x85EBCA6B) & _M32
    k ^= k >> 13
    k = (k * 0xC2B2AE35) & _M32
    k ^= k >> 16
    return k


def _murmur64(k):
    """hashmap.h:62-69 (Hash64Shift)."""
    k &= _M64
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & _M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & _M64
    k ^= k >> 33
    return k


def cache_hashmap_dir_size(total):
    """hashmap.cu:18 dir_size = _UpPower(total) * 2; _UpPower = 1 << (uint32)(log2(key) + 1),
    hashmap.h:91-94."""
    import math
    return (1 << int(math.log2(total) + 1)) * 2


def _home(key, cap, id_bytes):
    """hashmap.h:71-85: hash(int64 key) = (uint32)Hash64Shift(key) & (cap-1); int32: Hash32."""
    return (_murmur64(key) & _M32 if id_bytes == 8 else _murmur32(key)) & (cap - 1)


def cache_hashmap(lists, local_rank, id_bytes=8):
    """CreateNidsP2PCacheHashMapCUDA (hashmap.cu:15-77) executed sequentially: the remote ranks'
    lists in rotation order (index = (d + local_rank) % W), then the local list; each key by
    Hashmap::Update (hashmap.h:17-31: CAS at hash(key), then pos <- hash(pos + delta),
    delta = 1, 2, ..., value and device id written at the slot it holds).  Returns (key, idx,
    devid) int64 arrays of dir_size, -1 where empty.  (The reference inserts a list's keys
    concurrently: where two keys' probe chains meet, the slot each ends in depends on that
    order; this is the layout of one order, list order.)"""
    W = len(lists)
    total = sum(len(x) for x in lists)
    cap = cache_hashmap_dir_size(total)
    key = np.full(cap, -1, np.int64)
    idx = np.full(cap, -1, np.int64)
    dev = np.full(cap, -1, np.int64)
    order = [(d + local_rank) % W for d in range(W)]
    order = [i for i in order if i != local_rank] + [local_rank]
    for d in order:
        for i, k in enumerate(np.asarray(lists[d], np.int64).tolist()):
            pos, delta = _home(k, cap, id_bytes), 1
            while key[pos] != k and key[pos] != -1:
                pos = _murmur32(pos + delta) & (cap - 1)
                delta += 1
            key[pos] = k
            idx[pos] = i
            dev[pos] = d
    return key, idx, dev


def cache_hashmap_find(key, k, id_bytes=8):
    """Hashmap::SearchForPos (hashmap.h:33-47): the slot holding k, or -1."""
    cap = len(key)
    pos, delta = _home(int(k), cap, id_bytes), 1
    for _ in range(4 * cap):
        if key[pos] == k:
            return pos
        if key[pos] == -1:
            return -1
        pos = _murmur32(pos + delta) & (cap - 1)
        delta += 1
    return -1
