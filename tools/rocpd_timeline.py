"""Kernel timeline of the last dispatches in a rocprofv3 SQLite (rocpd) kernel trace: start
offset, duration and the idle gap before each kernel.

    python tools/rocpd_timeline.py gpurun_out/TAG_kt/run_results.db [LAST=60]
"""
import sqlite3
import sys


def main(db_path: str, last: int) -> None:
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()[-last:]
    t0 = rows[0][1]
    prev = t0
    for name, s, e in rows:
        name = name.replace("(anonymous namespace)::", "")
        name = name[5:] if name.startswith("void ") else name
        print(f"{(s - t0) / 1e6:9.3f} ms  {(e - s) / 1e6:8.3f} ms  gap {(s - prev) / 1e6:7.3f}  {name.split('(')[0][:80]}")
        prev = e
    print(f"span {(rows[-1][2] - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
