#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace database (rocpd SQLite) into a per-kernel CSV:
name, calls, mean/min/max/total duration (ns), VGPR/AGPR/LDS/scratch of the dispatch.

    python tools/prof_summary.py gpurun_out/prof/run_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys


def main(db: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), avg(duration), min(duration), max(duration), sum(duration),"
        " max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(scratch_size), max(grid_x)"
        " from kernels group by name order by sum(duration) desc").fetchall()
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "avg_ns", "min_ns", "max_ns", "total_ns", "vgpr", "agpr", "lds_bytes",
                "scratch_bytes", "grid_x"])
    for r in rows:
        w.writerow([r[0], r[1], round(r[2], 1), r[3], r[4], r[5], *r[6:]])


if __name__ == "__main__":
    main(sys.argv[1])
