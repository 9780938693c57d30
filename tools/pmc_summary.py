"""Summarize rocprofv3 outputs of a bench run into profiles/<tag>_summary.json.

Inputs (rocprofv3 --output-format csv):
  <dir>/<trace>_kernel_stats.csv            from --kernel-trace --stats
  <dir>/<fetch>_counter_collection.csv      from a separate --pmc FETCH_SIZE pass
  <dir>/<write>_counter_collection.csv      from a separate --pmc WRITE_SIZE pass
HBM traffic per dispatch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so
traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes.

usage: python tools/pmc_summary.py <dir> <tag> [trace fetch write]
"""
import collections
import csv
import json
import sys
from pathlib import Path


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").strip()


def main():
    d = Path(sys.argv[1])
    tag = sys.argv[2]
    trace, fetch, write = (sys.argv[3:6] if len(sys.argv) >= 6 else ("trace", "pmc_fetch", "pmc_write"))
    out = {"tag": tag, "kernels": {}}
    for r in csv.DictReader(open(d / f"{trace}_kernel_stats.csv")):
        n = short(r["Name"])
        if not n.startswith("llj::"):
            continue
        out["kernels"][n] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                             "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])}
    for fname, cname, key in ((fetch, "FETCH_SIZE", "fetch_kib"), (write, "WRITE_SIZE", "write_kib")):
        p = d / f"{fname}_counter_collection.csv"
        if not p.exists():
            continue
        agg = collections.defaultdict(list)
        seq = []
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == cname:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
                seq.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), float(r["Counter_Value"])))
        for n, v in agg.items():
            if n.startswith("llj::"):
                out["kernels"].setdefault(n, {})[key] = sum(v) / len(v)
        # the bench's dominant-kernel loop: >= 64 back-to-back dispatches of one GEMV kernel
        seq.sort()
        i = 0
        while i < len(seq):
            j = i
            while j < len(seq) and seq[j][1] == seq[i][1]:
                j += 1
            if j - i >= 64 and seq[i][1].startswith("llj::gemv"):
                lp = out.setdefault("dominant_loop", {}).setdefault(seq[i][1], {})
                lp.setdefault(key + "_list", []).extend(v for _, _, v in seq[i:j])
            i = j
    for n, lp in out.get("dominant_loop", {}).items():
        for key in ("fetch_kib", "write_kib"):
            v = lp.pop(key + "_list", None)
            if v:
                lp[key] = sum(v) / len(v)
                lp["dispatches"] = len(v)
        if "fetch_kib" in lp and "write_kib" in lp:
            lp["hbm_bytes_per_dispatch"] = (2 * lp["fetch_kib"] + lp["write_kib"]) * 1024
    for n, k in out["kernels"].items():
        if "fetch_kib" in k and "write_kib" in k:
            k["hbm_bytes_per_dispatch"] = (2 * k["fetch_kib"] + k["write_kib"]) * 1024
    tp = d / f"{trace}_kernel_trace.csv"
    if tp.exists():
        out.update(trace_phases(tp))
        for n, us in out["dominant_loop_avg_us"].items():
            out.setdefault("dominant_loop", {}).setdefault(n, {})["avg_us"] = us
    dst = Path(__file__).resolve().parent.parent / "profiles" / f"{tag}_summary.json"
    dst.write_text(json.dumps(out, indent=1, sort_keys=True))
    print(dst)


def trace_phases(path):
    """Per decode step (kernels between two greedy-argmax dispatches) kernel times, split by
    batch (attention grid Y = rows), and the bench's dominant-kernel loop (runs of >= 64
    back-to-back dispatches of one GEMV kernel = bench.py time_dominant_kernel)."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    steps = collections.defaultdict(list)
    cur = []
    for r in rows:
        n = short(r["Kernel_Name"])
        cur.append(r)
        if n == "llj::argmax_kernel":
            att = [x for x in cur if "attention" in x["Kernel_Name"]]
            if att and len(cur) > 20:
                steps[int(att[0]["Grid_Size_Y"])].append(cur)
            elif len(cur) > 20:  # chained layers (no standalone attention): batch from the argmax grid
                steps[int(r["Grid_Size_X"]) // 1024].append(cur)
            cur = []
    phases = {}
    for bsz, st in steps.items():
        # decode steps only: the most common kernel count (prefill / setup groups differ)
        mode = collections.Counter(len(s) for s in st).most_common(1)[0][0]
        st = [s for s in st if len(s) == mode]
        if len(st) < 4:
            continue
        st = st[2:]  # skip the first (warm-up / capture) steps
        per = collections.defaultdict(float)
        cnt = collections.defaultdict(int)
        span = []
        for s in st:
            span.append((int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3)
            for r in s:
                per[short(r["Kernel_Name"])] += dur(r)
                cnt[short(r["Kernel_Name"])] += 1
        phases[f"bs{bsz}"] = {"steps": len(st), "step_span_us": sum(span) / len(span),
                              "per_step_us": {k: v / len(st) for k, v in per.items()},
                              "avg_launch_us": {k: per[k] / cnt[k] for k in per}}
    loops = collections.defaultdict(list)
    i = 0
    while i < len(rows):
        j = i
        while j < len(rows) and rows[j]["Kernel_Name"] == rows[i]["Kernel_Name"]:
            j += 1
        if j - i >= 64 and short(rows[i]["Kernel_Name"]).startswith("llj::gemv"):
            loops[short(rows[i]["Kernel_Name"])] += [dur(r) for r in rows[i:j]]
        i = j
    return {"decode_steps": phases,
            "dominant_loop_avg_us": {k: sum(v) / len(v) for k, v in loops.items()}}


if __name__ == "__main__":
    main()
    raise SystemExit(0)
