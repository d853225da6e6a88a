"""ctypes binding of libdgs_amd.so (include/dgs_amd.h).

The library is the product: every op runs as HIP kernels on the current device.  There is
no CPU fallback -- if the shared object is missing or fails to load, importing `dgs`
raises.
"""
import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first; the library shares it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "DGS_AMD_LIB",
    os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libdgs_amd.so")))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"dgs: native library not found at {LIB_PATH}; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C dist-gnn_amd/csrc)")

lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)

c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_vp = ctypes.c_void_p
c_dbl = ctypes.c_double
p_i64 = ctypes.POINTER(ctypes.c_int64)
p_vp = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    "dgs_last_error": (ctypes.c_char_p, []),
    "dgs_version": (ctypes.c_char_p, []),
    "dgs_get_unique_id": (c_int, [p_i64]),
    "dgs_set_nccl": (c_int, [c_i64, p_i64, c_i64, c_i64]),
    "dgs_set_host_comm": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp]),
    "dgs_get_local_rank": (c_int, []),
    "dgs_get_world_size": (c_int, []),
    "dgs_barrier": (c_int, []),
    "dgs_allgather_sizes": (c_int, [c_i64, p_i64]),
    "dgs_allgather_bytes": (c_int, [c_vp, c_i64, p_vp, p_i64, c_vp]),
    "dgs_randn_uint64": (c_u64, []),
    "dgs_randn_uint64_n": (c_int, [c_i64, ctypes.POINTER(c_u64)]),
    "dgs_set_random_seed": (c_int, [c_u64]),
    "dgs_host_register": (c_int, [c_vp, c_i64]),
    "dgs_host_unregister": (c_int, [c_vp]),
    "dgs_host_registrations": (c_int, [c_i64, ctypes.POINTER(c_u64), p_i64, p_i64, p_i64,
                                       p_i64]),
    "dgs_host_memory_state": (c_int, [p_i64, p_i64, p_i64]),
    "dgs_abi_version": (c_int, []),
    "dgs_index_select": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_i64, c_vp, c_vp]),
    "dgs_index_select_device": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_i64, c_vp, c_vp]),
    "dgs_check_async_errors": (c_int, []),
    "dgs_last_gather_tag": (c_int, [ctypes.POINTER(c_u64)]),
    "dgs_stream_create": (c_int, [c_int, p_vp]),
    "dgs_stream_destroy": (c_int, [c_vp]),
    "dgs_stream_wait": (c_int, [c_vp, c_vp]),
    "dgs_stream_wait_event": (c_int, [c_vp, c_vp]),
    "dgs_sample_neighbors": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp,
                                     p_i64, c_vp]),
    "dgs_relabel": (c_int, [p_vp, p_i64, c_int, p_vp, p_i64, c_int, c_vp, p_i64, p_vp, c_vp]),
    "dgs_extract_indptr": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "dgs_extract_edge_data": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "dgs_test_bias_bounds": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "dgs_compute_frontier_heat": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                          c_i64, c_vp, c_vp]),
    "dgs_compute_frontier_heat_fixed": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                                c_i64, c_i64, c_vp, c_vp]),
    "dgs_p2p_server_create": (c_int, [c_vp, c_i64, c_i64, p_vp]),
    "dgs_p2p_server_device_ptr": (c_int, [c_vp, c_i64, p_vp, p_i64]),
    "dgs_p2p_server_destroy": (c_int, [c_vp]),
    "dgs_sampler_create": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, p_vp]),
    "dgs_sampler_bounds": (c_int, [c_vp, c_i64, p_i64, c_int, p_i64, p_i64]),
    "dgs_sampler_sample": (c_int, [c_vp, c_vp, c_i64, p_i64, c_int, c_int, p_vp, p_vp, p_vp,
                                   p_i64, c_vp]),
    "dgs_sampler_sample_packed": (c_int, [c_vp, c_vp, c_i64, p_i64, c_int, c_int, c_vp, p_i64,
                                          c_vp]),
    "dgs_sampler_sample_begin": (c_int, [c_vp, c_vp, c_i64, p_i64, c_int, c_int, p_vp, p_vp,
                                         p_vp, ctypes.POINTER(c_u64), c_int, c_vp]),
    "dgs_sampler_sample_end": (c_int, [c_vp, c_int, p_i64, c_vp]),
    "dgs_sampler_sample_packed_begin": (c_int, [c_vp, c_vp, c_i64, p_i64, c_int, c_int, c_vp,
                                                c_vp]),
    "dgs_sampler_sample_wait_hop": (c_int, [c_vp, c_int, c_int, p_i64, c_vp]),
    "dgs_sampler_sample_begin_after": (c_int, [c_vp, c_vp, c_vp, c_i64, p_i64, c_int, c_int,
                                               c_vp, ctypes.POINTER(c_u64), c_int, c_vp]),
    "dgs_loader_gather": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64,
                                  c_vp, c_i64, c_vp]),
    "dgs_sampler_context_count": (c_int, [c_vp, p_i64]),
    "dgs_sampler_local_cache": (c_int, [c_vp, p_vp, p_i64, p_vp, p_i64, p_vp]),
    "dgs_sampler_cache_hashmap_capacity": (c_int, [c_vp, p_i64]),
    "dgs_sampler_cache_hashmap_fill": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "dgs_sampler_cache_map_size": (c_int, [c_vp, p_i64]),
    "dgs_sampler_cache_map_fill": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "dgs_sampler_destroy": (c_int, [c_vp]),
    "dgs_feature_server_create": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, p_vp]),
    "dgs_feature_server_gather": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "dgs_feature_server_local_cache": (c_int, [c_vp, p_vp, p_i64]),
    "dgs_feature_server_layout": (c_int, [c_vp, ctypes.POINTER(c_int)]),
    "dgs_feature_server_destroy": (c_int, [c_vp]),
    "dgs_profile_enable": (c_int, [c_int]),
    "dgs_profile_read": (c_int, [ctypes.POINTER(c_dbl), p_i64, ctypes.POINTER(c_dbl), p_i64,
                                 ctypes.POINTER(c_dbl), p_i64]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = sorted(_SIGS)

ABI_VERSION = 6  # include/dgs_amd.h DGS_ABI_VERSION, the argument lists in _SIGS
if lib.dgs_abi_version() != ABI_VERSION:
    raise ImportError(f"dgs: {LIB_PATH} has ABI revision {lib.dgs_abi_version()}, this binding "
                      f"expects {ABI_VERSION}: rebuild the library")


def check(rc):
    if rc != 0:
        raise RuntimeError("dgs: " + lib.dgs_last_error().decode(errors="replace"))


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None):
    """Current HIP stream of `device` (torch.device, index or None = current device)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return c_vp(_raw_stream(idx))
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def i64_array(values):
    arr = (c_i64 * max(len(values), 1))(*[int(v) for v in values])
    return arr


def vp_array(values):
    return (c_vp * max(len(values), 1))(*[c_vp(int(v)) for v in values])
