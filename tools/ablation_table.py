"""Per-op in-graph kernel time of bs=8 decode under the GEMV ablation builds (tools/gpu_r04m.sh):
prod, abl1 (no A prologue), abl4 (minimal epilogue), abl7 (neither, no compute): prints one row per
decode op and the difference each ablation makes. usage: python tools/ablation_table.py <dir>"""
import csv
import sys
from pathlib import Path

OPS = {"void llj::gemv_kernel<0, 1, 3, 4, 4, 8, 3>": "swiglu", "void llj::gemv_kernel<0, 1, 2, 4, 4, 8, 3>": "qkv",
       "void llj::gemv_kernel<0, 0, 1, 8, 8, 8, 1>": "mlp.c_proj", "void llj::gemv_kernel<0, 1, 1, 4, 8, 8, 1>": "attn.c_proj"}


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        for pre, op in OPS.items():
            if r["Name"].startswith(pre):
                out[op] = float(r["AverageNs"]) / 1e3
    return out


d = Path(sys.argv[1])
vs = ["prod", "abl1", "abl4", "abl7"]
t = {v: load(d / f"{v}_kernel_stats.csv") for v in vs if (d / f"{v}_kernel_stats.csv").exists()}
print("op".ljust(12), *[v.rjust(8) for v in t])
for op in OPS.values():
    print(op.ljust(12), *[f"{t[v].get(op, float('nan')):8.2f}" for v in t])
