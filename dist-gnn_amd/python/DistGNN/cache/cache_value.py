"""Cache planner: which nodes' structure (sub-CSR) and feature rows each GPU keeps in HBM.

Counterpart of python/DistGNN/cache/cache_value.py:1-417 with the same functions, argument
names and return values, so example/graphsage/node_classification.py:13,46-151 runs unmodified.

Model (cache_value.py:155-206): a node's *heat* is the expected number of times a training
epoch touches it (sampling heat: its neighbour list is read; feature heat: its row is
gathered), propagated hop by hop with the `dgs` heat ops.  Caching a node saves
``heat * (read_bytes_host / bw_host - read_bytes_gpu / bw_gpu)`` of transfer time and costs its
bytes in HBM; nodes are taken greedily by value per byte until the free capacity is used.

* selfish  -- every GPU fills its own HBM with its own hottest nodes (cache_value.py:210-240);
* selfless -- every node is first offered to the GPU where it is hottest, lowest rank on ties
  (cache_value.py:64-150, 244-311); capacity left over is then filled selfishly.

MI355X differences (results identical): the owner of every node is found with two
all-reduces over the group (MAX of heat, then MIN of the ranks that hold that maximum) instead
of stacking all ranks' heat vectors on one GPU and scattering index lists back with
point-to-point sends -- on xGMI a ring all-reduce keeps every link busy, and no rank needs
W x N floats.  Sorts are stable so ties resolve by node order (deterministic plans);
`deterministic=True` in get_node_heat makes the heat itself order-independent.
"""
import torch
import torch.distributed as dist

import dgs

__all__ = [
    "get_node_heat", "get_hot_nids_local", "get_hot_nids_p2p_global", "get_structure_space",
    "get_feature_space", "get_node_value", "get_cache_nids_local", "get_cache_nids_selfish",
    "get_cache_nids_selfless", "compute_total_value_selfish", "compute_total_value_selfless",
    "get_available_memory",
]


# ------------------------------------------------------------------------------ heat
def get_node_heat(indptr, indices, node_ids, fan_outs, probs=None, mode="uva",
                  deterministic=False):
    """cache_value.py:6-53: per-node (sampling_heat, feature_heat) for the train nids.

    mode "uva" reads the host CSR zero-copy (pinned for the duration), "cuda" copies it to the
    GPU.  ADDITIVE deterministic=True: fixed-point heat accumulation (order-independent)."""
    if mode not in ("uva", "cuda"):
        raise ValueError("mode must be 'uva' or 'cuda'")
    host = (indptr, indices) + ((probs,) if probs is not None else ())
    if mode == "uva":
        for t in host:
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
            frontier_heat = dgs.ops._CAPI_compute_frontier_heat(
                seeds, indptr, indices, seeds_heat, k, 0, deterministic=deterministic)
        else:
            frontier_heat = dgs.ops._CAPI_compute_frontier_heat_with_bias(
                seeds, indptr, indices, probs, seeds_heat, k, 0, deterministic=deterministic)
        sampling_heat += seeds_heat
        seeds_heat += frontier_heat
        seeds = torch.nonzero(seeds_heat > 0).squeeze(1)
    feature_heat = sampling_heat + frontier_heat
    if mode == "uva":
        for t in host:
            dgs.ops._CAPI_tensor_unpin_memory(t)
    return sampling_heat, feature_heat


# ------------------------------------------------------------------------------ hot sets
def get_hot_nids_local(sampling_heat, feature_heat):
    """cache_value.py:57-60: every node with non-zero heat, in node order."""
    return torch.nonzero(sampling_heat).flatten(), torch.nonzero(feature_heat).flatten()


def _owned_nids(heat, group):
    """Nodes whose heat on this rank is the group maximum (lowest rank wins ties, as
    torch.argmax over the stacked heats) and non-zero here."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    top = heat.clone()
    dist.all_reduce(top, dist.ReduceOp.MAX, group)
    holder = torch.where(heat == top, torch.full_like(heat, rank, dtype=torch.int32),
                         torch.full_like(heat, world, dtype=torch.int32))
    dist.all_reduce(holder, dist.ReduceOp.MIN, group)
    nids = torch.nonzero(holder == rank).flatten()
    return nids[heat[nids] > 0]


def get_hot_nids_p2p_global(sampling_heat, feature_heat, group=None):
    """cache_value.py:64-150: nodes assigned to this GPU because it is where they are
    hottest (ascending node order)."""
    return _owned_nids(sampling_heat, group), _owned_nids(feature_heat, group)


# ------------------------------------------------------------------------------ cost model
def _no_probs(probs):
    # the reference's default is the *string* "None" (cache_value.py:153); both spellings mean
    # "no probability array"
    return probs is None or probs == "None"


def get_structure_space(nids, graph, probs="None"):
    """cache_value.py:153-167: HBM bytes of each node's cached neighbour list (+ probs) plus
    its indptr entry."""
    assert "indices" in graph and "indptr" in graph
    indptr = graph["indptr"].to(nids.device)
    deg = indptr[nids + 1] - indptr[nids]
    per_edge = graph["indices"].element_size()
    if not _no_probs(probs):
        assert probs in graph
        per_edge += graph[probs].element_size()
    return deg * per_edge + indptr.element_size()


def get_feature_space(graph):
    """cache_value.py:170-174: bytes of one feature row."""
    assert "features" in graph and "indptr" in graph
    feats = graph["features"]
    return int(feats.element_size() * feats.numel() / (graph["indptr"].numel() - 1))


def get_node_value(heat, space_bytes, reduced_time):
    """cache_value.py:178-181: time saved per byte of HBM."""
    assert isinstance(space_bytes, (int, torch.Tensor))
    return heat / space_bytes * reduced_time


def _reduced_time(bw_gpu, read_gpu, bw_host, read_host):
    return read_host / bw_host - read_gpu / bw_gpu


def _greedy_fill(value, cost, capacity):
    """Items by value (descending, stable), keeping the prefix whose running cost stays below
    capacity.  Returns (chosen item indices, running-cost array, number chosen)."""
    order = torch.argsort(value, descending=True, stable=True)
    running = torch.cumsum(cost[order], 0)
    cap = torch.tensor([capacity], device=running.device, dtype=running.dtype)
    n = int(torch.searchsorted(running, cap)[0])  # first position whose running cost >= cap
    return order[:n], running, n


def get_cache_nids_local(sampling_nids, sampling_space, sampling_value, feature_nids,
                         feature_space, feature_value, free_capacity_bytes):
    """cache_value.py:185-206: one greedy pass over structure and feature candidates
    together.  Returns (structure nids, feature nids, bytes used)."""
    ns = sampling_nids.numel()
    chosen, running, n = _greedy_fill(torch.cat([sampling_value, feature_value]),
                                      torch.cat([sampling_space, feature_space]),
                                      free_capacity_bytes)
    is_structure = chosen < ns
    structure = sampling_nids[chosen[is_structure]]
    feature = feature_nids[chosen[~is_structure] - ns]
    # bytes used: the running total at the last chosen item; with none chosen the reference
    # indexes position -1, i.e. reports the total of all candidates (kept: it makes the
    # selfless top-up below see no capacity left)
    used = running[n - 1].item() if running.numel() else 0
    return structure, feature, used


def _candidates(graph, nids_s, nids_f, sampling_heat, feature_heat, t_sampling, t_feature,
                probs):
    s_space = get_structure_space(nids_s, graph, probs=probs)
    s_value = get_node_value(sampling_heat[nids_s], s_space, t_sampling)
    f_row = get_feature_space(graph)
    f_value = get_node_value(feature_heat[nids_f], f_row, t_feature)
    return s_space, s_value, torch.full_like(nids_f, f_row), f_value


# ------------------------------------------------------------------------------ policies
def get_cache_nids_selfish(graph, sampling_heat, feature_heat, available_mem, bandwidth_gpu,
                           sampling_read_bytes_gpu, feature_read_bytes_gpu, bandwidth_host,
                           sampling_read_bytes_host, feature_read_bytes_host, probs=None):
    """cache_value.py:210-240: this GPU's own hottest nodes by value per byte."""
    t_s = _reduced_time(bandwidth_gpu, sampling_read_bytes_gpu, bandwidth_host,
                        sampling_read_bytes_host)
    t_f = _reduced_time(bandwidth_gpu, feature_read_bytes_gpu, bandwidth_host,
                        feature_read_bytes_host)
    nids_s, nids_f = get_hot_nids_local(sampling_heat, feature_heat)
    s_space, s_value, f_space, f_value = _candidates(graph, nids_s, nids_f, sampling_heat,
                                                     feature_heat, t_s, t_f, probs)
    s_nids, f_nids, _ = get_cache_nids_local(nids_s, s_space, s_value, nids_f, f_space,
                                             f_value, available_mem)
    return s_nids, f_nids


def get_cache_nids_selfless(graph, sampling_heat, feature_heat, available_mem, bandwidth_gpu,
                            sampling_read_bytes_gpu, feature_read_bytes_gpu, bandwidth_host,
                            sampling_read_bytes_host, feature_read_bytes_host, probs=None,
                            group=None):
    """cache_value.py:244-311: nodes owned by this GPU (hottest here) first; leftover
    capacity topped up selfishly with the other hot nodes; both lists ordered by heat."""
    t_s = _reduced_time(bandwidth_gpu, sampling_read_bytes_gpu, bandwidth_host,
                        sampling_read_bytes_host)
    t_f = _reduced_time(bandwidth_gpu, feature_read_bytes_gpu, bandwidth_host,
                        feature_read_bytes_host)
    own_s, own_f = get_hot_nids_p2p_global(sampling_heat, feature_heat, group=group)
    s_space, s_value, f_space, f_value = _candidates(graph, own_s, own_f, sampling_heat,
                                                     feature_heat, t_s, t_f, probs)
    s_nids, f_nids, used = get_cache_nids_local(own_s, s_space, s_value, own_f, f_space,
                                                f_value, available_mem)
    del own_s, own_f, s_space, s_value, f_space, f_value
    left = available_mem - used
    if left > 0:
        # the selfish pass must not pick what is already chosen: zero those heats in copies
        # (the reference zeroes and restores the caller's tensors in place)
        sh, fh = sampling_heat.clone(), feature_heat.clone()
        sh[s_nids] = 0
        fh[f_nids] = 0
        more_s, more_f = get_cache_nids_selfish(graph, sh, fh, left, bandwidth_gpu,
                                                sampling_read_bytes_gpu,
                                                feature_read_bytes_gpu, bandwidth_host,
                                                sampling_read_bytes_host,
                                                feature_read_bytes_host, probs=probs)
        del sh, fh
        s_nids = torch.cat([s_nids, more_s])
        f_nids = torch.cat([f_nids, more_f])
        s_nids = s_nids[torch.argsort(sampling_heat[s_nids], descending=True, stable=True)]
        f_nids = f_nids[torch.argsort(feature_heat[f_nids], descending=True, stable=True)]
    return s_nids, f_nids


# ------------------------------------------------------------------------------ plan value
def compute_total_value_selfish(graph, sampling_heat, feature_heat, sampling_cache_nids,
                                feature_cache_nids, bandwidth_gpu, sampling_read_bytes_gpu,
                                feature_read_bytes_gpu, bandwidth_host,
                                sampling_read_bytes_host, feature_read_bytes_host, probs=None):
    """cache_value.py:315-345: total time saved by a plan, every cached read local."""
    t_s = _reduced_time(bandwidth_gpu, sampling_read_bytes_gpu, bandwidth_host,
                        sampling_read_bytes_host)
    t_f = _reduced_time(bandwidth_gpu, feature_read_bytes_gpu, bandwidth_host,
                        feature_read_bytes_host)
    s_space = get_structure_space(sampling_cache_nids, graph, probs=probs)
    total = torch.sum(get_node_value(sampling_heat[sampling_cache_nids], s_space, t_s)).item()
    total += torch.sum(get_node_value(feature_heat[feature_cache_nids],
                                      get_feature_space(graph), t_f)).item()
    return total


def compute_total_value_selfless(graph, sampling_heat, feature_heat, sampling_cache_nids,
                                 feature_cache_nids, bandwidth_gpu, bandwidth_nvlink, num_gpu,
                                 sampling_read_bytes_gpu, feature_read_bytes_gpu,
                                 bandwidth_host, sampling_read_bytes_host,
                                 feature_read_bytes_host, probs=None, group=None):
    """cache_value.py:349-409: local reads at the HBM bandwidth left after the peers' share,
    plus the nodes other GPUs cache, read at the peer-link bandwidth (`bandwidth_nvlink`
    keeps the reference's name; on MI355X it is the per-peer xGMI rate)."""
    local_bw = bandwidth_gpu - (num_gpu - 1) * bandwidth_nvlink
    local = compute_total_value_selfish(graph, sampling_heat, feature_heat,
                                        sampling_cache_nids, feature_cache_nids, local_bw,
                                        sampling_read_bytes_gpu, feature_read_bytes_gpu,
                                        bandwidth_host, sampling_read_bytes_host,
                                        feature_read_bytes_host, probs=probs)
    n = graph["indptr"].numel() - 1
    dev = sampling_heat.device

    def elsewhere(mine):
        # nodes cached by some other rank: all-reduce of the membership masks (int32, not
        # bool, for every backend), then drop this rank's own
        m = torch.zeros(n, device=dev, dtype=torch.int32)
        m[mine] = 1
        dist.all_reduce(m, dist.ReduceOp.SUM, group)
        m[mine] = 0
        return torch.nonzero(m).flatten()

    remote = compute_total_value_selfish(graph, sampling_heat, feature_heat,
                                         elsewhere(sampling_cache_nids),
                                         elsewhere(feature_cache_nids), bandwidth_nvlink,
                                         sampling_read_bytes_gpu, feature_read_bytes_gpu,
                                         bandwidth_host, sampling_read_bytes_host,
                                         feature_read_bytes_host, probs=probs)
    return local + remote


def get_available_memory(device, reserved_mem):
    """cache_value.py:412-417: device memory (total, as the reference reads
    mem_get_info()[1]) minus what torch holds and a reserve; never negative."""
    total = torch.cuda.mem_get_info(device)[1]
    return max(int(total - torch.cuda.memory_allocated(device=device) - reserved_mem), 0)
