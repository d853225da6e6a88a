"""PMC calibration workload for the gather kernel: a sequential-row gather with a known byte
count (rows read once, in order), run under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
next to the bench so tools/pmc_traffic.py can derive the counter-to-bytes factor for the
kernel's own access pattern (MI355X_MICROARCH.md, HBM section)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dist-gnn_amd", "python"))
import torch  # noqa: E402

import dgs  # noqa: E402

N, REPS = 1 << 22, 5
D = int(os.environ.get("DGS_PMC_DIM", "100"))  # the bench's feature width
table = torch.randn(N, D, device="cuda")              # 1.68 GB, far beyond the 256 MB MALL
nids = torch.arange(N, dtype=torch.int64, device="cuda")
for _ in range(REPS):
    out = dgs.ops._CAPI_cuda_index_select(table, nids)
torch.cuda.synchronize()
print(f"calib rows={N} row_bytes={D * 4} reps={REPS}")
