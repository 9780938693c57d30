"""Prefill / perplexity-window throughput: LLaMA.forward over a (1, T) window
(no cache: every position's logits, as reference evaluate/full.py:118-125 calls it) on synthetic
7B weights (bench.build_model), for gptq.int4 and bf16. Prints one JSON line per (mode, T) with
the window time, tokens/s and the achieved dense FLOP/s of the Linear layers (2 * params * T)
over the whole forward; per-kernel times come from a rocprofv3 run of this script.

  python tools/prefill_bench.py [--T 512 2048] [--modes gptq.int4 none] [--iters 3]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402

if __import__("os").environ.get("LLJ_LIB"):  # an experiment build of the library (same ABI)
    sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
    from lit_llama import _hip  # noqa: E402

    _hip.LIB_PATH = Path(__import__("os").environ["LLJ_LIB"]).resolve()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", nargs="+", type=int, default=[512, 2048])
    ap.add_argument("--modes", nargs="+", default=["gptq.int4", "none"])
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--model", default="7B")
    ap.add_argument("--ab-w4z", type=int, default=0,
                    help="rounds of an interleaved A/B of the convert-once int4 GEMM (LLJ_OPT_GEMM_W4Z 1 vs 0)")
    ap.add_argument("--ab-flag", default=None,
                    help="NAME:ROUNDS -- interleaved A/B of a lit_llama.model module flag (True vs False), int4")
    a = ap.parse_args()
    if a.ab_w4z:
        return ab_w4z(a)
    if a.ab_flag:
        return ab_flag(a)
    for mode in a.modes:
        model = bench.build_model(a.model, None if mode == "none" else mode)
        cfg = model.config
        lin_params = sum(m.in_features * m.out_features for m in model.modules()
                         if hasattr(m, "in_features") and hasattr(m, "out_features"))
        for T in a.T:
            idx = torch.randint(3, cfg.vocab_size, (1, T), generator=torch.Generator().manual_seed(T)).cuda()
            with torch.no_grad():
                model(idx)  # warm-up (repack, attributes)
                torch.cuda.synchronize()
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for _ in range(a.iters):
                    model(idx)
                ev1.record()
                torch.cuda.synchronize()
            s = ev0.elapsed_time(ev1) / 1e3 / a.iters
            flops = 2.0 * lin_params * T
            print(json.dumps({"mode": mode, "model": a.model, "T": T, "ms_per_window": round(s * 1e3, 3),
                              "tokens_per_s": round(T / s, 1), "linear_tflops": round(flops / s / 1e12, 1),
                              "linear_mfma_frac_of_2.5PF": round(flops / s / 2.5e15, 4)}), flush=True)
        del model
        torch.cuda.empty_cache()



def ab_w4z(a):
    """Interleaved A/B in one process: the int4 window with the convert-once GEMM (option 1) and with
    the default int4 kernel (0), a.ab_w4z rounds of a.iters windows each; one JSON line per arm."""
    sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
    from lit_llama import _hip
    L = _hip.lib()
    model = bench.build_model(a.model, "gptq.int4")
    cfg = model.config
    for T in a.T:
        idx = torch.randint(3, cfg.vocab_size, (1, T), generator=torch.Generator().manual_seed(T)).cuda()
        res = {1: [], 0: []}
        with torch.no_grad():
            for arm in (1, 0):
                L.llj_set_option(_hip.OPT_GEMM_W4Z, arm)
                model(idx)  # warm-up per arm
            for _ in range(a.ab_w4z):
                for arm in (1, 0):
                    L.llj_set_option(_hip.OPT_GEMM_W4Z, arm)
                    torch.cuda.synchronize()
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record()
                    for _ in range(a.iters):
                        model(idx)
                    ev1.record()
                    torch.cuda.synchronize()
                    res[arm].append(ev0.elapsed_time(ev1) / a.iters)
        L.llj_set_option(_hip.OPT_GEMM_W4Z, -1)
        for arm in (1, 0):
            v = sorted(res[arm])
            print(json.dumps({"mode": "gptq.int4", "model": a.model, "T": T,
                              "arm": "convert-once (q - z) tile" if arm else "default int4 kernel",
                              "ms_per_window_median": round(v[len(v) // 2], 3), "ms_min": round(v[0], 3),
                              "rounds": a.ab_w4z}), flush=True)


def ab_flag(a):
    """Interleaved A/B in one process of a module flag of lit_llama.model (e.g. GEMM_SWIGLU), int4 window."""
    from lit_llama import model as MD
    name, rounds = a.ab_flag.split(":")
    model = bench.build_model(a.model, "gptq.int4")
    cfg = model.config
    for T in a.T:
        idx = torch.randint(3, cfg.vocab_size, (1, T), generator=torch.Generator().manual_seed(T)).cuda()
        res = {True: [], False: []}
        with torch.no_grad():
            for arm in (True, False):
                setattr(MD, name, arm)
                model(idx)
            for _ in range(int(rounds)):
                for arm in (True, False):
                    setattr(MD, name, arm)
                    torch.cuda.synchronize()
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record()
                    for _ in range(a.iters):
                        model(idx)
                    ev1.record()
                    torch.cuda.synchronize()
                    res[arm].append(ev0.elapsed_time(ev1) / a.iters)
        for arm in (True, False):
            v = sorted(res[arm])
            print(json.dumps({"mode": "gptq.int4", "model": a.model, "T": T, "flag": name, "arm": arm,
                              "ms_per_window_median": round(v[len(v) // 2], 3), "ms_min": round(v[0], 3),
                              "rounds": int(rounds)}), flush=True)


if __name__ == "__main__":
    main()
