"""Per-workgroup phase timeline of the decode GEMVs (profiling aid; a separate LLJ_TRACE build
of the library, never the product .so). Each GEMV workgroup stamps s_memrealtime (100 MHz) at
  0 start, 1 prologue + weight stream issued, 2 A image ready, 3 main loop done,
  4 wave partials reduced, 5 epilogue stored
(csrc/gemv_impl.h LLJ_STAMP). One eager decode step of 7B gptq.int4 bs=1 runs with a device
sync after every GEMV launch and its stamps are read back; prints, per op of one layer, the
median / p90 of each phase relative to the launch's first workgroup start.

  python tools/phase_trace.py [--build] [--layer 5] [--batch 1] [--quantize llm.int8] [--lib scratch/x.so]
  (--build [--defines LLJ_ABL=8 ...] --lib <out>: a trace build with extra macros)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
TRACE_SO = REPO / "scratch" / "lljamd_trace.so"

GEMV_CALLS = {"llj_norm_qkv_rope": "qkv", "llj_linear_resid": "resid", "llj_norm_swiglu": "swiglu",
              "llj_norm_linear": "head", "llj_i8_linear_resid": "resid", "llj_i8_swiglu_stats": "swiglu"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--layer", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--quantize", default="gptq.int4")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--defines", nargs="*", default=[])
    a = ap.parse_args()
    lib_path = REPO / a.lib if a.lib else TRACE_SO
    from lit_llama import _build, _hip

    if a.build:
        lib_path.parent.mkdir(exist_ok=True)
        _build.build(force=True, out=lib_path, defines=["LLJ_TRACE=1"] + a.defines)
        return
    _hip.LIB_PATH, _hip._lib = lib_path, None
    L = _hip.lib()
    copy = L.llj_trace_copy_i8 if a.quantize == "llm.int8" else L.llj_trace_copy_w4
    copy.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    import bench
    from lit_llama.engine import DecodeSession

    model = bench.build_model("7B", a.quantize)
    sess = DecodeSession(model, a.batch, 144, 120, use_graph=False)
    prompts = torch.randint(3, 32000, (a.batch, 16), generator=torch.Generator().manual_seed(0)).cuda()
    sess.prefill(prompts)
    sess.decode(40)
    torch.cuda.synchronize()
    buf = np.zeros(8192 * 8, np.uint64)
    records = []
    orig = _hip.call
    count = {}

    def spy(name, *args):
        orig(name, *args)
        if name in GEMV_CALLS:
            torch.cuda.synchronize()
            copy(buf.ctypes.data, buf.nbytes)
            count[name] = count.get(name, 0) + 1
            records.append((name, count[name], buf.reshape(8192, 8).copy()))
            buf[:] = 0
    _hip.call = spy
    sess.decode(1)
    torch.cuda.synchronize()
    _hip.call = orig
    out = {}
    per_layer = {"llj_norm_qkv_rope": 1, "llj_linear_resid": 2, "llj_norm_swiglu": 1, "llj_norm_linear": 1,
                 "llj_i8_linear_resid": 2, "llj_i8_swiglu_stats": 1}
    for name, k, tr in records:
        layer = (k - 1) // per_layer[name]
        if name != "llj_norm_linear" and layer != a.layer:
            continue
        tag = GEMV_CALLS[name] + ("" if GEMV_CALLS[name] != "resid" else ("_cproj" if (k - 1) % 2 == 0 else "_down"))
        ntiles = {"qkv": 768, "swiglu": 688, "head": 2000}.get(GEMV_CALLS[name], 256)
        tpw = 1
        if a.batch > 1 and a.quantize == "gptq.int4":  # multi-tile workgroups (pick_tpw: 256 CUs, <= 4; residual <= 2)
            tpw = min(4 if GEMV_CALLS[name] != "resid" else 2, -(-ntiles // 256))
        nwg = -(-ntiles // tpw)
        st = tr[:nwg, :6].astype(np.int64)
        valid = (st[:, 0] > 0) & (st[:, 5] >= st[:, 0])
        t0 = st[valid, 0].min()
        rel = (st[valid] - t0) * 10e-3  # us (100 MHz)
        res = {"workgroups": int(valid.sum()), "span_us": float(rel[:, 5].max())}
        for i, ph in enumerate(("start", "issued", "a_ready", "loop_done", "reduced", "stored")):
            res[ph] = {"med": round(float(np.median(rel[:, i])), 2), "p90": round(float(np.percentile(rel[:, i], 90)), 2),
                       "max": round(float(rel[:, i].max()), 2)}
        out[tag] = res
        print(tag, json.dumps(res), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    tag = f"{a.quantize}_bs{a.batch}" + (f"_{Path(a.lib).stem}" if a.lib else "")
    (REPO / "gpurun_out" / f"phase_trace_{tag}.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
