"""int8 GEMV layout probe (profiling aid): the LLM.int8 GEMV (CB in I8P tiles, wfmt 2) vs the gptq.int8
GEMV (W8P tiles, wfmt 3) on the same shapes, cold weights (8 copies > MALL), M = 1 / 8, no
outlier columns. python tools/w8_vs_i8.py"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
from lit_llama import _hip  # noqa: E402


def timed(run, n=200):
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda")
    L = _hip.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    NC = 8
    for (N, K) in [(4096, 4096), (4096, 11008), (11008, 4096)]:
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
        cb = torch.empty(N, K, dtype=torch.int8, device=dev)
        scb = torch.empty(N, dtype=torch.float32, device=dev)
        _hip.call("llj_i8_quant_weight", W.data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st)
        cbr = cb.clone()
        _hip.call("llj_i8_repack", cbr.data_ptr(), cb.data_ptr(), N, K, st)  # the GEMV reads the I8P tiling
        cbs = [cb.clone() for _ in range(NC)]
        # gptq.int8: random codes in the reference layout -> W8P
        qref = torch.randint(0, 256, (K, N), dtype=torch.uint8, device=dev, generator=g)
        w8 = [torch.empty(N * K, dtype=torch.uint8, device=dev) for _ in range(NC)]
        for t in w8:
            _hip.call("llj_w8_repack", qref.data_ptr(), t.data_ptr(), N, K, st)
        sc = torch.full((N,), 0.01, device=dev)
        zr = torch.full((N,), 128.0, device=dev)
        sz = torch.empty(N, 2, dtype=torch.float32, device=dev)
        _hip.call("llj_w8_scale_zero", sc.data_ptr(), zr.data_ptr(), 0, sz.data_ptr(), N, st)
        del W
        for M in (1, 8):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            ws = torch.empty(L.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
            _hip.call("llj_i8_stats", x.data_ptr(), K, M, K, 6.0, ws.data_ptr(), st)
            y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            it = [0]

            def run_i8():
                c = cbs[it[0] % NC]
                it[0] += 1
                _hip.call("llj_linear", 2, x.data_ptr(), K, c.data_ptr(), scb.data_ptr(), None, y.data_ptr(), N, M, N,
                          K, ws.data_ptr(), 0, None, st)

            def run_w8():
                c = w8[it[0] % NC]
                it[0] += 1
                _hip.call("llj_linear", 3, x.data_ptr(), K, c.data_ptr(), sz.data_ptr(), None, y.data_ptr(), N, M, N,
                          K, None, 0, None, st)
            for name, run in (("llm.int8 CB (I8P tiles)", run_i8), ("gptq.int8 W8P", run_w8)):
                us = timed(run)
                print(json.dumps({"N": N, "K": K, "M": M, "kernel": name, "us": round(us, 2),
                                  "GBps": round(N * K / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
