"""The half-wave lane moves of dist-gnn_amd/csrc/dgs_lane.cuh (DPP and v_permlane16_swap in
place of ds_bpermute in the top-k networks of the biased kernels) against HIP's __shfl forms on
the GPU: tools/lane_ops_test (built by __graft_entry__.build() with the library)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_lane_moves_match_shuffles():
    exe = os.path.join(ROOT, "tools", "lane_ops_test")
    assert os.path.exists(exe), "tools/lane_ops_test is built by __graft_entry__.build()"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "lane ops: ok" in out.stdout, out.stdout + out.stderr
