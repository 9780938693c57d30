"""Timing of the int8 (LLM.int8) GEMV (llj_linear_resid, wfmt 2) at the 7B shapes and bs 1 / 8,
by outlier regime of the activation: none; SURVEY section 8(d)'s C3 regime (6 of the K columns
scaled x20); 40 and 300 columns x25 (the synthetic-weight model's own range). Weights cycle through
8 copies (> the 256 MB MALL). Prints one JSON line per case: python tools/i8_bench.py"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
from lit_llama import _hip  # noqa: E402


def main():
    dev = torch.device("cuda")
    L = _hip.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    NC = 8  # weight copies streamed in turn (> the 256 MB MALL): every launch reads cold weights
    for (N, K) in [(4096, 11008), (4096, 4096), (12288, 4096)]:
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
        cb = torch.empty(N, K, dtype=torch.int8, device=dev)
        scb = torch.empty(N, dtype=torch.float32, device=dev)
        _hip.call("llj_i8_quant_weight", W.data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st)
        cbr = cb.clone()
        _hip.call("llj_i8_repack", cbr.data_ptr(), cb.data_ptr(), N, K, st)  # the GEMV reads the I8P tiling
        cbs = [cb] + [cb.clone() for _ in range(NC - 1)]
        del W
        for M in (1, 8):
            for nout, mult in ((0, 1), (6, 20), (40, 25), (300, 25)):
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
                x.clamp_(-5.5, 5.5)  # no accidental outliers (|x| >= 6.0) outside the injected columns
                if nout:
                    cols = torch.randperm(K, device=dev, generator=g)[:nout]
                    x[:, cols] *= mult
                ws = torch.empty(L.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
                y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
                _hip.call("llj_i8_stats", x.data_ptr(), K, M, K, 6.0, ws.data_ptr(), st)

                it = [0]

                def run():
                    c = cbs[it[0] % NC]
                    it[0] += 1
                    _hip.call("llj_linear_resid", 2, x.data_ptr(), K, c.data_ptr(), scb.data_ptr(), y.data_ptr(), N,
                              M, N, K, ws.data_ptr(), 0, None, st)
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(200):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 200
                print(json.dumps({"N": N, "K": K, "M": M, "outlier_cols": nout, "outlier_mult": mult,
                                  "us": round(us, 2), "GBps": round((N * K + 4 * N + 2 * M * (K + 2 * N)) / us / 1e3, 1),
                                  "frac_of_8TBs": round((N * K + 4 * N + 2 * M * (K + 2 * N)) / us / 1e3 / 8000, 3)}),
                      flush=True)


if __name__ == "__main__":
    main()
