"""Decode throughput of every BASELINE.json config on one MI355X (the bench line covers C2/bs8).

  C1  LLaMA-7B bf16 (unquantized), bs=1
  C2  LLaMA-7B gptq.int4, bs=1 and bs=8
  C3  LLaMA-7B llm.int8, bs=8, in three outlier regimes of the Linear inputs (bench.build_model):
      the random weights' own (C3), none (C3-o0) and SURVEY §8d's 6 columns x20 (C3-o6x20)
  C4  LLaMA-13B gptq.int4, bs=1 (one replica; the driver runs the 8-replica scan)
  X-gptq.int8  LLaMA-7B gptq.int8 (ColBlock bits=8), bs=1 (not a BASELINE config; informational)
  C2-long      LLaMA-7B gptq.int4, bs=1 with a 1900-token prompt in a 2048-slot cache (SURVEY §8d's
               long-KV point; split-K attention)

Synthetic weights of the exact shapes (bench.build_model), 16-token random prompts,
max_seq_length 144, greedy; value = decode tokens/s, step_roofline = algorithmic bytes of a
step / step time / 8 TB/s.

usage: python tools/config_suite.py [--out FILE] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import gc
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402

CONFIGS = [("C1", "7B", "none", 1), ("C2", "7B", "gptq.int4", 1), ("C2-bs8", "7B", "gptq.int4", 8),
           ("C2-long", "7B", "gptq.int4", 1),
           ("C3", "7B", "llm.int8", 8), ("C3-o0", "7B", "llm.int8", 8), ("C3-o6x20", "7B", "llm.int8", 8),
           ("C4", "13B", "gptq.int4", 1),
           ("X-gptq.int8", "7B", "gptq.int8", 1)]  # extra: the reference's third --quantize mode
LONG = {"C2-long": (1900, 2048)}  # (prompt length, max_seq_length)
OUTLIERS = {"C3-o0": "none", "C3-o6x20": "6x20"}  # bench.build_model's llm.int8 outlier regimes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--only", default=None, help="comma-separated config tags")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    results = []
    models = {}
    for tag, name, mode, B in CONFIGS:
        if a.only and tag not in a.only.split(","):
            continue
        key = (name, mode, OUTLIERS.get(tag))
        if key not in models:
            models.clear()
            gc.collect()
            torch.cuda.empty_cache()
            models[key] = bench.build_model(name, None if mode == "none" else mode, outliers=OUTLIERS.get(tag))
        model = models[key]
        plen, S = LONG.get(tag, (16, 144))
        r = bench.time_decode(model, B, plen, S, a.warmup, min(a.steps, 2048 - plen - 1 - a.warmup), 1)
        sb = bench.step_bytes(model, B, r["pos_mean"])
        t_step = r["seconds"] / (r["tokens"] // B)
        line = {"config": tag, "model": f"LLaMA-{name}", "quantize": mode, "outliers": OUTLIERS.get(tag, "random weights"),
                "batch": B, "prompt_len": plen,
                "max_seq_length": S,
                "value": round(r["tokens"] / r["seconds"], 2), "unit": "tokens/s",
                "ms_per_step": round(t_step * 1e3, 4), "bytes_per_step": sb,
                "step_roofline": {"achieved_GBps": round(sb / t_step / 1e9, 1),
                                  "frac": round(sb / t_step / 1e9 / bench.HBM_PEAK_GBS, 4)},
                "data": f"synthetic weights of the exact shapes, random {plen}-token prompts, greedy"}
        del r["session"]
        print(json.dumps(line), flush=True)
        results.append(line)
    if a.out:
        Path(a.out).write_text(json.dumps(results, indent=1))


if __name__ == "__main__":
    main()
