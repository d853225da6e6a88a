"""tools/pmc_traffic.py on synthetic rocprofv3 counter CSVs (no GPU): per-row HBM bytes come from
each launch's grid, launches far larger than the bench's own (the 2^20-row micro-benchmark in
the same run) are left out, and the read factor comes from the calibration gather."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_traffic  # noqa: E402

GATHER = "void dgs::(anonymous namespace)::k_gather<16, dgs::(anonymous namespace)::StridedSrc<false> >(x)"
PLAIN = "void dgs::(anonymous namespace)::k_gather<16, dgs::(anonymous namespace)::PlainSrc<long> >(x)"


def _csv(path, counter, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        for name, grid, kib in rows:
            w.writerow([name, grid, counter, kib])


def _grid(rows, row_bytes=400):
    # one-wave workgroups of 64 lanes x 4 chunks of 16 B
    return int(rows * (row_bytes // 16) / 4)


def test_bytes_per_row_from_grids(tmp_path):
    root = str(tmp_path)
    bench_rows, big_rows = 100_000, 1 << 20
    # bench launches: 520 B read and 400 B written per row; micro-bench launches: 2x the bytes
    # per row (must not move the result)
    rd = [(GATHER, _grid(bench_rows), bench_rows * 520 / 2 / 1024)] * 5
    rd += [(GATHER, _grid(big_rows), big_rows * 1040 / 2 / 1024)] * 2
    wr = [(GATHER, _grid(bench_rows), bench_rows * 400 / 1024)] * 5
    wr += [(GATHER, _grid(big_rows), big_rows * 800 / 1024)] * 2
    _csv(f"{root}/pmc_bench_fetch/run/x_counter_collection.csv", "FETCH_SIZE", rd)
    _csv(f"{root}/pmc_bench_write/run/x_counter_collection.csv", "WRITE_SIZE", wr)
    n = 1 << 22
    _csv(f"{root}/pmc_calib_fetch/run/x_counter_collection.csv", "FETCH_SIZE",
         [(PLAIN, 0, n * 408 / 2 / 1024)])  # FETCH_SIZE sees half of a coalesced stream
    _csv(f"{root}/pmc_calib_write/run/x_counter_collection.csv", "WRITE_SIZE",
         [(PLAIN, 0, n * 400 / 1024)])
    with open(f"{root}/pmc_bench_fetch.log", "w") as f:
        f.write(json.dumps({"gathered_rows_per_step": bench_rows}) + "\n")
    out = pmc_traffic.main(root)
    assert out["bench_launches"] == 5 and out["launches_left_out"] == 2
    assert abs(out["calibration"]["read_factor"] - 2.0) < 1e-9
    assert abs(out["hbm_read_bytes_per_row"] - 520) < 1e-6
    assert abs(out["hbm_write_bytes_per_row"] - 400) < 1e-6
    assert abs(out["hbm_bytes_per_launch"] - 920 * bench_rows) < 1e-3
