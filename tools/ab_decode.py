"""A/B timing of decode-step variants that are switched by module-level flags of
lit_llama.model (e.g. ATTN_RESID), on the bench workload (synthetic 7B weights, 16-token
prompt, S = 144). Variants are interleaved (rounds x variants) in one process on the same
weights, so box-to-box and clock drift cancel. Prints one JSON line per (variant, batch).

  python tools/ab_decode.py --variants base:ATTN_RESID=0 fused:ATTN_RESID=1 --batch 1 8
A variant may also name another build of the library (same ABI, e.g. other -D macros):
  python tools/ab_decode.py --variants base d8:LIB=scratch/d8.so
and the host-side knobs TPW (llj_set_tpw_max) and STREAM (llj_set_stream_a).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))

import bench  # noqa: E402
from lit_llama import model as MD  # noqa: E402


def parse_variant(spec: str):
    name, _, assigns = spec.partition(":")
    flags = {}
    for a in filter(None, assigns.split(",")):
        k, v = a.split("=")
        flags[k] = v if k == "LIB" else (int(v) if v.lstrip("-").isdigit() else (v == "True"))
    return name, flags


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--batch", nargs="+", type=int, default=[1])
    ap.add_argument("--model", default="7B")
    ap.add_argument("--quantize", default="gptq.int4")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--max-seq-length", type=int, default=144)
    args = ap.parse_args()
    mode = None if args.quantize == "none" else args.quantize
    model = bench.build_model(args.model, mode)
    variants = [parse_variant(v) for v in args.variants]
    from lit_llama import _hip

    default_lib = _hip.LIB_PATH
    defaults = {k: getattr(MD, k) for _, f in variants for k in f if k not in ("LIB", "TPW", "STREAM", "SPECB")}
    res = {(n, b): [] for n, _ in variants for b in args.batch}
    for r in range(args.rounds):
        for b in args.batch:
            for name, flags in variants:
                for k, v in defaults.items():
                    setattr(MD, k, v)
                lib = Path(flags.get("LIB", default_lib))
                if not lib.is_absolute():
                    lib = REPO / lib
                if _hip.LIB_PATH != lib:  # experiment variant of the library (same ABI)
                    _hip.LIB_PATH, _hip._lib = lib, None
                _hip.lib().llj_set_tpw_max(int(flags.get("TPW", 4)))
                _hip.lib().llj_set_stream_a(int(flags.get("STREAM", 1)))
                _hip.lib().llj_set_option(_hip.OPT_ATT_SPEC_BATCH, int(flags.get("SPECB", -1)))
                for k, v in flags.items():
                    if k not in ("LIB", "TPW", "STREAM", "SPECB"):
                        setattr(MD, k, v)
                t = bench.time_decode(model, b, 16, args.max_seq_length, 5, args.steps, 1)
                ms = t["gpu_seconds"] / args.steps * 1e3
                res[(name, b)].append(ms)
                print(f"[ab] round {r} {name} bs={b}: {ms:.4f} ms/step", file=sys.stderr, flush=True)
                del t
    for (name, b), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"variant": name, "batch": b, "ms_per_step": round(med, 4), "all": [round(x, 4) for x in v],
                          "tokens_per_s": round(b / med * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
