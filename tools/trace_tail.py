"""Per-kernel average duration over the LAST n dispatches of a rocprofv3 kernel trace (the timed
decode steps of tools/ab_decode.py / bench.py come last; the prompt prefill, whose int8 slices
carry thousands of outlier columns, comes first and would dominate a whole-run average).
  python tools/trace_tail.py <kernel_trace.csv> [n] > summary.json"""
from __future__ import annotations

import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8000
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-n:]
    agg = collections.defaultdict(list)
    for r in tail:
        agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    out = {"dispatches": len(tail), "span_us": round(span, 1),
           "kernels": sorted(({"name": k[:110], "calls": len(v), "avg_us": round(sum(v) / len(v), 3),
                               "total_us": round(sum(v), 1)} for k, v in agg.items()), key=lambda d: -d["total_us"])}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
