"""Prompt-GEMM epilogue probe: the 7B QKV GEMM (M = 2048, N = 12288, K = 4096, integral-zero int4) timed as
llj_gemm_qkv_rope (RoPE + q / KV-cache stores) and as llj_gemm_linear (plain bf16 store) on the same weights,
plus the window's other int4 GEMMs (mlp c_proj residual, N = 4096, K = 11008; the one-pass SwiGLU, H = 11008),
interleaved; prints one JSON line. Timing only (random codes, scales, zeros 8)."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
from lit_llama import _hip  # noqa: E402


def main():
    L = _hip.lib()
    dev = "cuda"
    M, C, nh, S = 2048, 4096, 32, 2048
    N, K = 3 * C, C
    g = torch.Generator(device=dev).manual_seed(5)
    qw = torch.randint(0, 256, (K // 2, N), dtype=torch.uint8, device=dev, generator=g)
    Wp = torch.empty_like(qw)
    _hip.call("llj_w4_repack", qw.data_ptr(), Wp.data_ptr(), N, K, 0)
    sc = torch.full((N,), 0.002, dtype=torch.float32, device=dev)
    zr = torch.full((N,), 8.0, dtype=torch.float32, device=dev)
    sz = torch.empty(N, 2, dtype=torch.float32, device=dev)
    _hip.call("llj_w4_scale_zero", sc.data_ptr(), zr.data_ptr(), 0, sz.data_ptr(), N, 0)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    q = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.empty(1, nh, S, C // nh, dtype=torch.bfloat16, device=dev)
    vc = torch.empty_like(kc)
    rope = torch.randn(S, C // nh // 2, 2, device=dev, generator=g)
    pos = torch.arange(M, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    wf = _hip.WF_ZINT

    def w4(n, k):
        qw = torch.randint(0, 256, (k // 2, n), dtype=torch.uint8, device=dev, generator=g)
        wp = torch.empty_like(qw)
        _hip.call("llj_w4_repack", qw.data_ptr(), wp.data_ptr(), n, k, 0)
        s = torch.empty(n, 2, dtype=torch.float32, device=dev)
        _hip.call("llj_w4_scale_zero", torch.full((n,), 0.002, device=dev).data_ptr(),
                  torch.full((n,), 8.0, device=dev).data_ptr(), 0, s.data_ptr(), n, 0)
        return wp, s

    H = 11008
    Wd, szd = w4(C, H)
    W1, s1 = w4(H, C)
    W2, s2 = w4(H, C)
    hx = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
    xr = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    hh = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    nb = L.llj_gemm_swiglu_ws_bytes(wf, M, H, K)
    ws = torch.empty(max(nb, 4) // 4, dtype=torch.float32, device=dev)
    runs = {
        "qkv_rope": lambda: _hip.call("llj_gemm_qkv_rope", wf, x.data_ptr(), Wp.data_ptr(), sz.data_ptr(), q.data_ptr(),
                                      kc.data_ptr(), vc.data_ptr(), rope.data_ptr(), pos.data_ptr(), 1, M, C, nh, S, st),
        "store": lambda: _hip.call("llj_gemm_linear", wf, x.data_ptr(), K, Wp.data_ptr(), sz.data_ptr(), out.data_ptr(), N,
                                   M, N, K, st),
        "resid_c_proj": lambda: _hip.call("llj_gemm_resid", wf, hx.data_ptr(), H, Wd.data_ptr(), szd.data_ptr(),
                                          xr.data_ptr(), C, M, C, H, st),
        "swiglu": lambda: _hip.call("llj_gemm_swiglu", wf, x.data_ptr(), K, W1.data_ptr(), s1.data_ptr(), W2.data_ptr(),
                                    s2.data_ptr(), hh.data_ptr(), H, M, H, K, st),
        "swiglu_ws": lambda: _hip.call("llj_gemm_swiglu_ws", wf, x.data_ptr(), K, W1.data_ptr(), s1.data_ptr(),
                                       W2.data_ptr(), s2.data_ptr(), hh.data_ptr(), H, M, H, K, ws.data_ptr(), nb, st),
    }
    res = {k: [] for k in runs}
    for f in runs.values():
        f()
    torch.cuda.synchronize()
    for _ in range(5):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(json.dumps({k: round(sorted(v)[2], 1) for k, v in res.items()} | {"unit": "us per launch (median of 5 x 10)",
                                                                              "shape": [M, N, K]}))


if __name__ == "__main__":
    main()
