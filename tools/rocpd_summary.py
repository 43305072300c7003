"""Summarise a rocprofv3 SQLite (rocpd) kernel trace into a per-kernel stats CSV.

    python tools/rocpd_summary.py gpurun_out/prof27/run_results.db profiles/r01b_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db_path: str, out_path: str) -> None:
    db = sqlite3.connect(db_path)
    rows = db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(workgroup_x), max(lds_size), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "pct", "grid_threads",
                    "workgroup", "lds_bytes", "vgpr", "agpr", "sgpr"])
        for r in rows:
            name = r[0].replace("(anonymous namespace)::", "")
            name = name[5:] if name.startswith("void ") else name
            name = name.split("(")[0]
            w.writerow([name, r[1], int(r[2]), int(r[3]), int(r[4]), int(r[5]), round(100.0 * r[2] / total, 4)] +
                       list(r[6:]))
    print(open(out_path).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
