"""Tensor plumbing for the ctypes binding: dtype checks, device views of library memory."""
import torch

from ._lib import c_vp

_TYPESTR = {
    torch.int64: "<i8", torch.int32: "<i4", torch.float32: "<f4", torch.float64: "<f8",
    torch.float16: "<f2", torch.bfloat16: "<V2", torch.uint8: "|u1", torch.int8: "|i1",
    torch.int16: "<i2", torch.bool: "|b1",
}


class _CudaArray:
    """__cuda_array_interface__ exporter for a non-owning view of library device memory."""

    def __init__(self, ptr, shape, dtype, owner):
        self.__cuda_array_interface__ = {
            "shape": tuple(int(s) for s in shape), "typestr": _TYPESTR[dtype],
            "data": (int(ptr), False), "version": 2, "strides": None,
        }
        self._owner = owner


def device_view(ptr, shape, dtype, owner, device=None):
    """Non-owning CUDA tensor over `ptr` (the library block stays alive via `owner`),
    like the reference's torch::from_blob views (tensor_p2p_cache.cc:120-132)."""
    numel = 1
    for s in shape:
        numel *= int(s)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    if numel == 0 or not ptr:
        return torch.empty(tuple(shape), dtype=dtype, device=dev)
    if dtype == torch.bfloat16:
        t = torch.as_tensor(_CudaArray(ptr, shape, torch.int16, owner), device=dev)
        return t.view(torch.bfloat16)
    return torch.as_tensor(_CudaArray(ptr, shape, dtype, owner), device=dev)


def ptr(t):
    return c_vp(t.data_ptr()) if t is not None and t.numel() > 0 else c_vp(0)


def as_i64(t, name):
    if t.dtype not in (torch.int32, torch.int64):
        raise RuntimeError(f"{name}: ID can only be int32 or int64")
    return t.to(torch.int64).contiguous() if t.dtype != torch.int64 else t.contiguous()


def check_cuda(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


def check_cpu(t, name):
    if t.is_cuda:
        raise RuntimeError(f"{name} must be a CPU tensor")


def row_bytes(t):
    stride = 1
    for s in t.shape[1:]:
        stride *= int(s)
    return stride, stride * t.element_size()
