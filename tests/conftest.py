import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_test_drained(request):
    """After every GPU test: collect garbage (services finalised in GC cycles are destroyed
    here, not inside a later test), drain the device and check the library's async error
    report.  A fault or an out-of-range gather is then attributed to the test that caused it
    (an asynchronous HIP error otherwise surfaces at whatever call comes next)."""
    yield
    if "gpu" not in request.keywords:
        return
    import gc
    import torch
    if not torch.cuda.is_available():
        return
    gc.collect()
    torch.cuda.synchronize()
    import dgs
    dgs.ops._check_async_errors()
    # No library registration outlives its users: the only registrations are the pins
    # _CAPI_tensor_pin_memory still holds (services copy pageable arrays instead, DESIGN.md
    # section 3), so once those are dropped the table is empty.  The table goes into the report.
    regs = dgs.ops._host_registrations()
    pinned = {base for _, base in dgs.ops._registered.values()}
    stray = [r for r in regs if r["base"] not in pinned]
    assert not stray, f"host registrations outlived their users: {regs}"
