"""Summarize round-2 rocprofv3 outputs (kernel trace + separate PMC passes) into one small JSON.

Reads from <dir>:
  trace_kernel_trace.csv / trace_kernel_stats.csv        --kernel-trace --stats of bench.py
  <tag>_counter_collection.csv                           one --pmc pass each (eager decode)
Per kernel (llj:: kernels only, grouped by name + grid size), the per-dispatch average of every
counter, and derived:
  hbm_bytes   = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (MI355X_MICROARCH.md §HBM gfx950 correction)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
                (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs x 4 SIMDs)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  mfma_tflops = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / profiled duration
For the 7B gptq.int4 bs=1 kernels, the algorithmic bytes per launch and the
PMC traffic / algorithmic ratio. usage: python tools/profile_summary.py <dir> <out.json>
"""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import trace_phases  # noqa: E402

C, H, V = 4096, 11008, 32000


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").strip()


def op_of(name: str, grid: int, multi: bool = False) -> str | None:
    """7B decode op of a gemv instantiation (template args WF, AM, EP, NW, D, MB, TPW) by grid;
    multi: the run's decode rows are batched (bs=8 passes), so MB = 8 forms are decode ops."""
    if not name.startswith("llj::gemv_kernel<"):
        return None
    a = [int(x) for x in name[len("llj::gemv_kernel<"):-1].split(",")]
    ep, nw, mb = a[2], a[3], a[5]
    if mb != 1 and not multi:
        # a multi-row instantiation in the bs=1 run is a prompt slice (8 rows of the 16-token
        # prompt): its second slice reads the weights back from the 256 MB MALL, so its HBM bytes
        # fall below the algorithmic bytes (the round-2 "0.809x" row) -- not a decode op
        return None
    wgs = grid // (nw * 64)
    if ep == 2:
        return "qkv"
    if ep == 3:
        return "swiglu"
    if ep == 0:
        return "lm_head"
    if ep == 1:
        return "mlp.c_proj" if nw == 8 else "attn.c_proj"
    return None


def algo_bytes_int4(op: str, M: int = 1) -> float:
    """packed codes + bf16 (scale, zero) per row + activations in / out."""
    def lin(N, K):
        return N * K / 2 + 4 * N
    return {"qkv": lin(3 * C, C) + M * C * 2 + M * 3 * C * 2,
            "attn.c_proj": lin(C, C) + M * C * 2 + 2 * M * C * 2,
            "swiglu": 2 * lin(H, C) + M * C * 2 + M * H * 2,
            "mlp.c_proj": lin(C, H) + M * H * 2 + 2 * M * C * 2,
            "lm_head": lin(V, C) + M * C * 2 + M * V * 2}[op]


def algo_bytes_int8(op: str, M: int = 1) -> float:
    """LLM.int8 GEMV (wfmt 2): int8 CB codes + fp32 SCB + the quantized rows (int8) + bf16 out / residual."""
    def lin(N, K):
        return N * K + 4 * N
    return {"qkv": lin(3 * C, C) + M * C + M * 3 * C * 2,
            "attn.c_proj": lin(C, C) + M * C + 2 * M * C * 2,
            "swiglu": 2 * lin(H, C) + M * C + M * H * 2,
            "mlp.c_proj": lin(C, H) + M * H + 2 * M * C * 2,
            "lm_head": lin(V, C) + M * C + M * V * 2}[op]


def main():
    d = Path(sys.argv[1])
    out = {"source": str(d), "passes": {}, "kernels": {}}
    groups = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for p in sorted(d.glob("*_counter_collection.csv")):
        tag = p.name[:-len("_counter_collection.csv")]
        names = set()
        for r in csv.DictReader(open(p)):
            n = short(r["Kernel_Name"])
            if not n.startswith("llj::"):
                continue
            key = f"{tag}|{n}|{r['Grid_Size']}"
            groups[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            names.add(r["Counter_Name"])
            durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        out["passes"][tag] = sorted(names)
    for key, cs in groups.items():
        tag, n, grid = key.split("|")
        prefix = tag.split("_")[0]  # bs1 / bs8 / c1 / c3 / c3b8 (int8 bs=8 decode in 4-row slices) / c3h
        op = op_of(n, int(grid), multi=prefix in ("bs8", "c3b8", "c3", "c3h"))
        if prefix == "c3h" and op:  # the C++ harness at one C3 shape per run: the op is in the tag
            op = {"qkv": "qkv", "head": "lm_head", "swiglu": "swiglu", "cproj": "attn.c_proj",
                  "down": "mlp.c_proj"}.get(tag.split("_")[1], op)
            prefix = "c3h_" + tag.split("_")[1]
        k = out["kernels"].setdefault(f"{n} grid {grid}" + (f" ({prefix})" if prefix.startswith("c3h") else ""), {"op": op})
        ent = k.setdefault(prefix, {})
        ent["dispatches"] = max(ent.get("dispatches", 0), max(len(v) for v in cs.values()))
        for c, v in cs.items():
            ent[c] = sum(v) / len(v)
        ent.setdefault("profiled_us", sum(durs[key]) / len(durs[key]))
    for name, k in out["kernels"].items():
        for prefix, ent in list(k.items()):
            if not isinstance(ent, dict):
                continue
            if "FETCH_SIZE" in ent and "WRITE_SIZE" in ent:
                ent["hbm_bytes"] = (2 * ent["FETCH_SIZE"] + ent["WRITE_SIZE"]) * 1024
                if prefix in ("bs1", "bs8") and k["op"]:
                    ent["algorithmic_bytes"] = algo_bytes_int4(k["op"], 8 if prefix == "bs8" else 1)
                    ent["traffic_over_algorithmic"] = round(ent["hbm_bytes"] / ent["algorithmic_bytes"], 3)
                elif (prefix in ("c3", "c3b8") or prefix.startswith("c3h")) and k["op"] and name.startswith("llj::gemv_kernel<2,"):
                    ent["algorithmic_bytes"] = algo_bytes_int8(k["op"], 4 if prefix == "c3b8" else 8)
                    ent["traffic_over_algorithmic"] = round(ent["hbm_bytes"] / ent["algorithmic_bytes"], 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in ent and ent.get("GRBM_GUI_ACTIVE"):
                ent["mfma_busy"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (ent["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if "SQ_WAIT_ANY" in ent and ent.get("SQ_WAVE_CYCLES"):
                ent["wait_frac"] = ent["SQ_WAIT_ANY"] / ent["SQ_WAVE_CYCLES"]
            if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in ent:
                ent["mfma_tflops_profiled"] = ent["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / (ent["profiled_us"] * 1e-6) / 1e12
    tp = d / "trace_kernel_trace.csv"
    if tp.exists():
        out.update(trace_phases(tp))
    Path(sys.argv[2]).write_text(json.dumps(out, indent=1, sort_keys=True))
    print(sys.argv[2])


if __name__ == "__main__":
    main()
