"""Per-kernel statistics (the rocprofv3 --stats kernel table: Name, Calls, TotalNs, AverageNs, MinNs, MaxNs,
Percentage) from a rocprofv3 rocpd SQLite output (run_results.db, the default output format of this
image's rocprofv3), for committing under profiles/ next to the csv summaries of earlier rounds.

  python tools/kstats_db.py gpurun_out/r06b/prof8 > profiles/r06b_bs8_kernel_stats.csv
"""
from __future__ import annotations

import csv
import glob
import sqlite3
import sys
from collections import defaultdict


def kernel_rows(path: str):
    dbs = glob.glob(f"{path}/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    rows = defaultdict(list)
    for db in dbs:
        c = sqlite3.connect(db)
        names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
        kd = [n for n in names if n.startswith("rocpd_kernel_dispatch")]
        ks = [n for n in names if n.startswith("rocpd_info_kernel_symbol")]
        for d, s in zip(sorted(kd), sorted(ks)):
            q = f"select k.kernel_name, d.end - d.start from {d} d join {s} k on d.kernel_id = k.id"
            for name, dur in c.execute(q):
                rows[name].append(dur)
    return rows


def main():
    rows = kernel_rows(sys.argv[1])
    total = sum(sum(v) for v in rows.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100 * sum(v) / total, 3), min(v), max(v)])


if __name__ == "__main__":
    main()
