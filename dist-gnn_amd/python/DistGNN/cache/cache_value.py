"""Cache planning counterpart (python/DistGNN/cache/cache_value.py) -- heat propagation
over the MI355X `dgs` heat ops.  (Selection policies: see DESIGN.md, section "Next".)"""
import torch

import dgs

__all__ = ["get_node_heat"]


def get_node_heat(indptr, indices, node_ids, fan_outs, probs=None, mode="uva"):
    """cache_value.py:6-53: per-node sampling / feature heat for the given train nids."""
    if mode not in ("uva", "cuda"):
        raise ValueError("mode must be 'uva' or 'cuda'")
    if mode == "uva":
        for t in (indptr, indices) + ((probs,) if probs is not None else ()):
            dgs.ops._CAPI_tensor_pin_memory(t)
    else:
        indptr, indices = indptr.cuda(), indices.cuda()
        probs = probs.cuda() if probs is not None else None
    n = indptr.shape[0] - 1
    sampling_heat = torch.zeros(n, device="cuda")
    seeds_heat = torch.zeros(n, device="cuda")
    seeds_heat[node_ids] = 1
    seeds = node_ids.cuda()
    frontier_heat = torch.zeros(n, device="cuda")
    for k in reversed(fan_outs):
        if probs is None:
            frontier_heat = dgs.ops._CAPI_compute_frontier_heat(seeds, indptr, indices,
                                                                seeds_heat, k, 0)
        else:
            frontier_heat = dgs.ops._CAPI_compute_frontier_heat_with_bias(
                seeds, indptr, indices, probs, seeds_heat, k, 0)
        sampling_heat += seeds_heat
        seeds_heat += frontier_heat
        seeds = torch.nonzero(seeds_heat > 0).squeeze(1)
    feature_heat = sampling_heat + frontier_heat
    if mode == "uva":
        for t in (indptr, indices) + ((probs,) if probs is not None else ()):
            dgs.ops._CAPI_tensor_unpin_memory(t)
    return sampling_heat, feature_heat
