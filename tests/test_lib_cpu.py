"""CPU-side checks of the native library (no GPU needed): it loads, exports every symbol
include/dgs_amd.h declares, and its launch-seed engine matches the oracle's mt19937_64."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dgs_amd.h")
LIB = os.path.join(ROOT, "dist-gnn_amd", "lib", "libdgs_amd.so")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char \*|int|uint64_t)\s*(dgs_\w+)\(", src,
                                 re.M)))


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"


def test_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (dgs_\w+)", out))
    declared = _declared()
    assert len(declared) >= 30
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_binding_covers_declared_symbols():
    import dgs
    assert sorted(dgs._lib.EXPORTED) == _declared()


def test_binding_mirrors_reference_module_layout():
    import dgs
    ops = {"_CAPI_get_unique_id", "_CAPI_set_nccl", "_CAPI_compute_frontier_heat",
           "_CAPI_compute_frontier_heat_with_bias", "_CAPI_tensor_pin_memory",
           "_CAPI_tensor_unpin_memory", "_CAPI_cuda_sample_neighbors",
           "_CAPI_cuda_sample_neighbors_bias", "_CAPI_cuda_sampled_tensor_relabel",
           "_CAPI_cuda_index_select", "_Test_Randn", "_Test_NCCLTensorAllGather",
           "_Test_GetLocalRank", "_Test_GetWorldSize", "_Test_ExtractEdgeData",
           "_Test_ExtractIndptr"}
    assert ops <= set(dir(dgs.ops))
    for cls, methods in {
            "P2PCacheSampler": ["_CAPI_sample_node_classifiction",
                                "_CAPI_get_cpu_structure_tensors",
                                "_CAPI_get_local_cache_structure_tensors",
                                "_CAPI_get_local_cache_hashmap_tensors"],
            "P2PCacheFeatureServer": ["_CAPI_get_cpu_feature", "_CAPI_get_gpu_feature",
                                      "_CAPI_get_feature"],
            "TensorP2PServer": ["_CAPI_get_device_tensor", "_CAPI_get_local_device_tensor"]}.items():
        c = getattr(dgs.classes, cls)
        for m in methods:
            assert callable(getattr(c, m)), (cls, m)
    import DistGNN
    assert DistGNN.capi is dgs


def test_launch_seed_engine_matches_oracle():
    import dgs
    from oracle import oracle as O
    dgs.ops._CAPI_set_random_seed(20261015)
    got = [dgs.ops._Test_Randn() for _ in range(6)]
    assert got == O.launch_seeds(20261015, 6)


def test_world_defaults_before_set_nccl():
    import dgs
    assert dgs.ops._Test_GetLocalRank() == 0
    assert dgs.ops._Test_GetWorldSize() == 1


def test_seed_generator():
    import torch
    from DistGNN.dataloading import SeedGenerator
    data = torch.arange(10)
    batches = list(SeedGenerator(data, 4))
    assert [b.tolist() for b in batches] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
    assert len(list(SeedGenerator(data, 4, drop_last=True))) == 2
    torch.manual_seed(0)
    got = torch.cat(list(SeedGenerator(data, 3, shuffle=True)))
    assert sorted(got.tolist()) == list(range(10))


@pytest.mark.parametrize("scale,ef", [(8, 4), (10, 8)])
def test_rmat_generator_shape(scale, ef):
    import numpy as np
    from DistGNN.dataloading.synthetic import rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(scale, ef)
    assert indptr.size == (1 << scale) + 1 and indices.size == (1 << scale) * ef
    assert indptr[-1] == indices.size and (np.diff(indptr) >= 0).all()
    assert indices.min() >= 0 and indices.max() < (1 << scale)
