"""Derives per-launch HBM traffic of the feature-gather kernel from rocprofv3 PMC CSVs.

Inputs: counter_collection CSVs of four runs -- {bench, calibration} x {FETCH_SIZE,
WRITE_SIZE} (separate passes: FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2).  FETCH_SIZE /
WRITE_SIZE are in KiB.  The read-side factor comes from the calibration run (sequential
gather of known bytes, same kernel, 16-B lane loads) -- on gfx950 FETCH_SIZE reads about 1/2
of a wide coalesced stream's bytes (MI355X_MICROARCH.md, HBM).
Writes profiles/gather_pmc.json (read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import sys


def unroll_of(name):
    """16-B chunks per lane of a gather launch: the kernel's second template argument since
    round 5 (k_gather<16, 8, ...> for large gathers), 4 before."""
    import re
    m = re.search(r"k_gather<16, (\d+), ", name)
    return int(m.group(1)) if m else 4


def per_kernel(path_glob, counter, kernel_re, with_grid=False):
    import re
    vals = []
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            if re.search(kernel_re, name):
                v = float(r["Counter_Value"])
                vals.append((v, int(r.get("Grid_Size", 0) or 0) * unroll_of(name))
                            if with_grid else v)
    return vals


def rows_of_grid(grid_chunks_per_lane, row_bytes, vec=16, threads=64):
    """Rows of one gather launch from its grid size times the launch's chunks per lane
    (one-wave workgroups; the fused label workgroups, at most a few dozen, are within the
    rounding)."""
    return max(1.0, grid_chunks_per_lane / (row_bytes / vec))


def bench_side(fetch, write, row_bytes):
    """Per-row HBM bytes over the bench's own gathers: launches whose grid says they gathered
    more than 4x the median rows (the 2^20-row micro-benchmark in the same run) are left out."""
    def per_row(vals):
        rows = [rows_of_grid(g, row_bytes) for _, g in vals]
        med = sorted(rows)[len(rows) // 2]
        keep = [(v, r) for (v, _), r in zip(vals, rows) if r <= 4 * med]
        return sum(v for v, _ in keep) * 1024 / sum(r for _, r in keep), len(keep), len(vals)
    return per_row(fetch), per_row(write)


def kernel_names(path_glob):
    names = set()
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            names.add(r.get("Kernel_Name", ""))
    return names


def main(root):
    # the feature-server gather: computed addresses (StridedSrc, whole graph cached) or the
    # address-table form (TableSrc)
    table_re = (r"k_gather<16, (\d+, )?dgs::\(anonymous namespace\)::"
                r"(TableSrc|StridedSrc<\w+>) ?>")
    plain_re = r"k_gather<16, (\d+, )?dgs::\(anonymous namespace\)::PlainSrc<long> >"
    bf = per_kernel(f"{root}/pmc_bench_fetch/**/*counter_collection.csv", "FETCH_SIZE", table_re,
                    with_grid=True)
    bw = per_kernel(f"{root}/pmc_bench_write/**/*counter_collection.csv", "WRITE_SIZE", table_re,
                    with_grid=True)
    cf = per_kernel(f"{root}/pmc_calib_fetch/**/*counter_collection.csv", "FETCH_SIZE", plain_re)
    cw = per_kernel(f"{root}/pmc_calib_write/**/*counter_collection.csv", "WRITE_SIZE", plain_re)
    assert bf and bw and cf and cw, (len(bf), len(bw), len(cf), len(cw))
    kernel_name = "k_gather<16, StridedSrc>" if any(
        "StridedSrc" in n for n in kernel_names(f"{root}/pmc_bench_fetch/**/*counter_collection.csv")
    ) else "k_gather<16, TableSrc>"
    N, D = 1 << 22, int(os.environ.get("DGS_PMC_DIM", "100"))
    calib_read = N * (D * 4 + 8)          # rows + nids
    calib_write = N * D * 4
    cfetch = sorted(cf)[len(cf) // 2] * 1024
    cwrite = sorted(cw)[len(cw) // 2] * 1024
    read_factor = calib_read / cfetch
    write_factor = calib_write / cwrite
    bench_rows = float(os.environ.get("BENCH_ROWS_PER_LAUNCH", "0"))
    line = glob.glob(f"{root}/pmc_bench_fetch.log")
    if not bench_rows and line:
        for ln in open(line[0]):
            if ln.startswith("{"):
                bench_rows = json.loads(ln)["gathered_rows_per_step"]
    (rd_row, n_kept, n_all), (wr_row, _, _) = bench_side(bf, bw, D * 4)
    rd_row *= read_factor
    wr_row *= write_factor
    fetch = rd_row * bench_rows if bench_rows else None
    write = wr_row * bench_rows if bench_rows else None
    out = {
        "kernel": kernel_name, "dim": D,
        "calibration": {"workload": f"sequential gather of 2^22 rows x {D * 4} B (tools/gather_calib.py)",
                        "expected_read_bytes": calib_read, "fetch_size_bytes": cfetch,
                        "read_factor": read_factor, "expected_write_bytes": calib_write,
                        "write_size_bytes": cwrite, "write_factor": write_factor},
        "bench_launches": n_kept,
        "launches_left_out": n_all - n_kept,
        "rows_per_launch_source": "each launch's grid size (micro-benchmark launches left out)",
        "hbm_read_bytes_per_row": rd_row, "hbm_write_bytes_per_row": wr_row,
        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": (fetch + write) if bench_rows else None,
        "rows_per_launch": bench_rows or None,
        "hbm_bytes_per_row": rd_row + wr_row,
    }
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    res = main(sys.argv[1])
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
