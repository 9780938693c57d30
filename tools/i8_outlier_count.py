"""Outlier-column counts of every llj_i8_stats call of a 7B llm.int8 decode (profiling aid)."""
import sys, json, collections
from pathlib import Path; R = Path(__file__).resolve().parent.parent; sys.path.insert(0, str(R)); sys.path.insert(0, str(R / "lit-llama-ja_amd"))
import torch, bench
from lit_llama import _hip
model = bench.build_model("7B", "llm.int8")
orig = _hip.call
stats = collections.defaultdict(list)
def call(name, *a):
    r = orig(name, *a)
    if name == "llj_i8_stats":
        ws_ptr, M, K = a[5], a[2], a[3]
        torch.cuda.synchronize()
        kb = ((K + 31) // 32 + 15) & ~15
        off_cnt = 16 + 4 * 32 * M
        buf = torch.empty(off_cnt + 4 * 32, dtype=torch.uint8, device="cuda")
        import ctypes
        hipMemcpy = ctypes.CDLL("libamdhip64.so").hipMemcpy
        host = (ctypes.c_int * 32)()
        hipMemcpy(host, ctypes.c_void_p(ws_ptr + off_cnt), ctypes.c_size_t(128), 3)
        stats[(M, K)].append(sum(host))
    return r
_hip.call = call
for b in (1, 8):
    stats.clear()
    bench.time_decode(model, b, 16, 144, 1, 3, 1, use_graph=False)
    print(json.dumps({"batch": b, **{f"M{k[0]}_K{k[1]}": [min(v), int(sum(v)/len(v)), max(v)] for k, v in stats.items()}}), flush=True)
