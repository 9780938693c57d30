"""GPTQ producer timing at LLaMA-7B Linear shapes (synthetic fp32 weights and calibration rows):
whole GPTQQuantizer.quantize() per Linear, the llj_gptq_block column-loop kernel alone (HIP events
on its stream), and the numpy oracle on a bounded row sample of the same K (CPU companion,
scaled to all rows). One JSON line per shape.

  python tools/gptq_bench.py [--tokens 8192] [--cpu-rows 256]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))

from lit_llama import _hip  # noqa: E402
from lit_llama.quantization import GPTQQuantizer  # noqa: E402

SHAPES = {"c_attn": (12288, 4096), "c_proj": (4096, 4096), "c_fc1": (11008, 4096), "mlp.c_proj": (4096, 11008)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192, help="calibration rows fed through the hook")
    ap.add_argument("--cpu-rows", type=int, default=256)
    args = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, K) in SHAPES.items():
        lin = torch.nn.Linear(K, N, bias=False, device=dev)
        lin.weight.data = torch.randn(N, K, device=dev, generator=g) * 0.02
        gq = GPTQQuantizer(lin, bits=4, groupsize=-1, actorder=True)
        h = lin.register_forward_hook(gq.collect_input_stats)
        x = torch.randn(args.tokens // 2048, 2048, K, device=dev, generator=g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            for j in range(x.shape[0]):
                lin(x[j:j + 1])
        torch.cuda.synchronize()
        t_hook = time.perf_counter() - t0
        h.remove()
        H = gq.H.clone()
        t0 = time.perf_counter()
        qm, err = gq.quantize()
        torch.cuda.synchronize()
        t_quant = time.perf_counter() - t0
        # the column-loop kernel alone, every block of the Linear, on the quantizer's operands
        Hd = H + 0.01 * torch.mean(torch.diag(H)) * torch.eye(K, device=dev)
        Hinv = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hd)), upper=True).contiguous()
        Wt = lin.weight.detach().t().contiguous()
        Qt, Err = torch.empty_like(Wt), torch.empty(128, N, device=dev)
        loss = torch.zeros(N, device=dev)
        sc = torch.rand(N, device=dev) * 0.01 + 1e-3
        zr = torch.full((N,), 8.0, device=dev)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(s)
        for _ in range(reps):
            for i1 in range(0, K, 128):
                _hip.call("llj_gptq_block", Hinv.data_ptr(), K, i1, Wt.data_ptr(), N, sc.data_ptr(), zr.data_ptr(), 4,
                          Qt.data_ptr(), Err.data_ptr(), loss.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        launches = reps * (K // 128)
        us = e0.elapsed_time(e1) * 1e3 / launches
        # per launch: the block's weights in + reconstructions and errors out (fp32), Hinv1 per workgroup
        nbytes = 3 * N * 128 * 4 + ((N + 127) // 128) * 128 * 128 * 4
        flops = 2 * N * (128 * 127 // 2)  # one multiply + one subtract per triangular update
        # CPU companion: the oracle on a row sample of the same K (column loop + trailing update)
        from oracle import gptq_np as G
        rows = min(args.cpu_rows, N)
        Wc = lin.weight.detach()[:rows].cpu().numpy()
        Hc = H.cpu().numpy()
        t0 = time.perf_counter()
        G.gptq_quantize(Wc, Hc, 4)
        t_cpu = (time.perf_counter() - t0) * N / rows
        print(json.dumps({
            "linear": name, "N": N, "K": K, "calib_tokens": args.tokens, "hook_s": round(t_hook, 4),
            "quantize_s": round(t_quant, 4), "block_kernel_us": round(us, 2),
            "block_kernel_GBps": round(nbytes / us / 1e3, 1), "block_kernel_TFLOPs": round(flops / us / 1e6, 3),
            "cpu_oracle_s_scaled": round(t_cpu, 2), "cpu_sample_rows": rows, "error": round(err, 3)}), flush=True)
        del lin, gq, qm, x, H, Hinv, Wt, Qt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
