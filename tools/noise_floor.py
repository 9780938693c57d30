"""bf16 noise floor of the 7B / 13B-width parity tests (tests/test_model_7b_gpu.py): the oracle
against ITSELF with every Linear summed in another valid order, on the tests' own weights, ids and
teacher-forced steps. The oracle rounds to bf16 at the reference's points, so any two correct
implementations differ by 1-ulp bf16 flips that then propagate through the layers; this measures
how large that difference gets at these shapes, i.e. the smallest tolerance a parity test against
this oracle can honestly use.

Orders compared, per Linear y = x W^T (W dequantized for gptq.int4):
  base   numpy float32 matmul (BLAS blocking; the tests' oracle)
  f64    float64 accumulation, rounded to float32 once (as exact as fp32 output allows)
  chunk  float32 sums of 128-deep K chunks added in chunk order (the GPU GEMV's K chunking)
and the fp32 mean of every bf16 RMSNorm (model.py:281) taken in the same order. LLM.int8's int32
GEMM is exact in every order; its dequantization product SCA * SCB / 127^2 * acc (float64 / another
association) and its fp16 outlier side product take the alternative orders.

Usage: python tools/noise_floor.py [--out profiles/r03_noise_floor.json]  (CPU, a few minutes)
       python tools/noise_floor.py --generic [--out profiles/r03_noise_floor_generic.json]
         the any-shape configs of tests/test_generic_gpu.py (reference test n_embd 32 x 16 layers,
         3 x 64 rows no-cache; 125M prompt rows + decode steps, bf16 and gptq.int4)
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from oracle import llama_np as O  # noqa: E402
from tests import test_model_7b_gpu as T  # noqa: E402  (weights / ids / steps of the parity tests)

F32 = np.float32


class AltLinear:
    """A Linear of the oracle evaluated in another summation order."""

    def __init__(self, spec: O.LinearSpec, order: str):
        self.spec, self.order = spec, order
        if spec.kind == "dense":
            self.w = spec.w.astype(F32)
        elif spec.kind == "colblock":
            self.w = O.colblock_get_weight(spec.qw, spec.scales, spec.zeros, spec.bits)
        else:
            self.w = None
        self._w64 = None

    def _mm(self, x, w):
        if self.order == "f64":
            if self._w64 is None or self._w64.shape != w.shape:
                self._w64 = w.astype(np.float64)
            return (x.astype(np.float64) @ self._w64.T).astype(F32)
        K = x.shape[-1]
        acc = np.zeros(x.shape[:-1] + (w.shape[0],), F32)
        for k0 in range(0, K, 128):
            acc = (acc + (x[..., k0:k0 + 128].astype(F32) @ w[:, k0:k0 + 128].T)).astype(F32)
        return acc

    def __call__(self, x):
        if self.w is not None:
            return self._mm(x.astype(F32), self.w)
        s = self.spec  # LLM.int8: exact int32 part + the fp16 side product in this order
        A = x.astype(F32).reshape(-1, x.shape[-1])
        a16 = A.astype(np.float16).astype(F32)
        big = np.abs(a16) >= 6.0
        outl = np.nonzero(big.any(axis=0))[0]
        inl = np.where(big, F32(0.0), a16)
        sca = np.abs(inl).max(axis=1).astype(F32)
        safe = np.where(sca == 0, F32(1.0), sca)
        ca = np.rint(inl * (F32(127.0) / safe[:, None])).clip(-127, 127)
        ca[:, outl] = 0
        acc = ca.astype(np.float64) @ s.cb.astype(np.float64).T
        if self.order == "f64":  # the dequant product in float64, rounded once
            out = (acc * (sca[:, None].astype(np.float64) * s.scb[None, :] / (127.0 * 127.0))).astype(F32)
        else:  # the same product associated as (acc * SCA) * (SCB / 127^2)
            out = ((acc.astype(F32) * sca[:, None]) * (s.scb[None, :] / F32(127.0 * 127.0))).astype(F32)
        if outl.size:
            wsub = (s.cb[:, outl].astype(F32) * (s.scb[:, None] / F32(127.0))).astype(np.float16).astype(F32)
            out = out + (a16[:, outl].astype(np.float64) @ wsub.T.astype(np.float64)).astype(F32)
        return out.reshape(*x.shape[:-1], s.cb.shape[0]).astype(F32)


class AltOracle(O.OracleLLaMA):
    """The oracle with its Linears and its RMSNorm means summed in `order`."""

    def __init__(self, cfg, pb, lin, order):
        super().__init__(cfg, pb, linears=lin, act_bf16=True)
        self.order = order
        self.lin = {k: AltLinear(v, order) for k, v in self.lin.items()}

    def _norm(self, x, scale):  # oracle.rmsnorm_bf16 with the mean in `order`
        r16 = O.bf16_round
        x = r16(x)
        xx = r16(x * x)
        C = x.shape[-1]
        if self.order == "f64":
            ms = (xx.astype(np.float64).sum(-1, keepdims=True) / C).astype(F32)
        else:
            acc = np.zeros(x.shape[:-1] + (1,), F32)
            for k0 in range(0, C, 128):
                acc = (acc + xx[..., k0:k0 + 128].sum(-1, keepdims=True, dtype=F32)).astype(F32)
            ms = (acc / F32(C)).astype(F32)
        ms = r16(ms)
        e = r16(ms + F32(1e-5))
        r = r16(F32(1.0) / np.sqrt(e))
        return r16(r16(scale.astype(F32)) * r16(x * r))


def orc_variant(cfg, pb, lin, order):
    if order == "base":
        return O.OracleLLaMA(cfg, pb, linears=lin, act_bf16=True)
    return AltOracle(cfg, pb, lin, order)


def rels(a, b):
    return [float(np.linalg.norm(a[i, s] - b[i, s]) / np.linalg.norm(b[i, s]))
            for i in range(a.shape[0]) for s in range(a.shape[1])]


def _case(name, outs):
    case = {"case": name, "rel_base_vs_f64": rels(outs["base"], outs["f64"]),
            "rel_base_vs_chunk": rels(outs["base"], outs["chunk"]), "rel_f64_vs_chunk": rels(outs["f64"], outs["chunk"])}
    case["floor_max"] = max(max(case[k]) for k in case if k.startswith("rel_"))
    case["floor_mean"] = float(np.mean([v for k in case if k.startswith("rel_") for v in case[k]]))
    print(f"[noise] {name}: floor max {case['floor_max']:.3e} mean {case['floor_mean']:.3e}", flush=True)
    return case


def generic_cases():
    from tests import test_generic_gpu as TG

    cases = []
    cfg = TG.REF_TEST
    pb, _, lin = T.oracle_linears(T.make_params(cfg, 32), None)
    idx = np.random.default_rng(3).integers(0, cfg.vocab_size, (3, 64))
    cases.append(_case("ref-test n_embd 32 x16 no-cache 3x64 rows",
                       {o: orc_variant(cfg, pb, lin, o).forward(idx) for o in ("base", "f64", "chunk")}))
    cfg = TG.C125
    p = T.make_params(cfg, 125)
    ids = np.random.default_rng(12).integers(3, cfg.vocab_size, (2, 12 + 5))
    for mode in (None, "gptq.int4"):
        pb, _, lin = T.oracle_linears(p, mode)
        outs_rows, outs_steps = {}, {}
        for o in ("base", "f64", "chunk"):
            st, rows = T._oracle_steps(orc_variant(cfg, pb, lin, o), ids, t_prompt=12, steps=4, s=32, all_rows=True)
            outs_rows[o], outs_steps[o] = rows, st
        cases.append(_case(f"125M {mode} prompt rows", outs_rows))
        cases.append(_case(f"125M {mode} steps", outs_steps))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--widths", default="4096,5120")
    ap.add_argument("--generic", action="store_true")
    args = ap.parse_args()
    res = {"what": __doc__.split("\n\n")[0], "cases": []}
    if args.generic:
        res["cases"] = generic_cases()
        out = args.out or str(REPO / "profiles" / "r03_noise_floor_generic.json")
        Path(out).write_text(json.dumps(res, indent=1))
        print(f"wrote {out}")
        return
    args.out = args.out or str(REPO / "profiles" / "r03_noise_floor.json")
    for width in [int(w) for w in args.widths.split(",")]:
        cfg = T.C7 if width == 4096 else T.C13
        p = T.make_params(cfg, T.SEEDS[width])
        modes = ["gptq.int4", None, "llm.int8"] if width == 4096 else ["gptq.int4"]
        for mode in modes:
            pb, _, lin = T.oracle_linears(p, mode)
            rng_seed = (1 + 17) if width == 4096 else (1 + 31)  # the tests' B = 1 ids
            ids = np.random.default_rng(rng_seed).integers(3, cfg.vocab_size, (1, T.T_PROMPT + T.STEPS + 1))
            outs = {}
            for order in ("base", "f64", "chunk"):
                t0 = time.time()
                outs[order] = T._oracle_steps(orc_variant(cfg, pb, lin, order), ids)
                print(f"[noise] width {width} {mode} {order}: {time.time() - t0:.1f} s", flush=True)
            case = {"width": width, "mode": str(mode), "batch": 1, "steps": T.STEPS + 1,
                    "rel_base_vs_f64": rels(outs["base"], outs["f64"]),
                    "rel_base_vs_chunk": rels(outs["base"], outs["chunk"]),
                    "rel_f64_vs_chunk": rels(outs["f64"], outs["chunk"])}
            case["floor_max"] = max(max(case[k]) for k in case if k.startswith("rel_"))
            case["floor_mean"] = float(np.mean([v for k in case if k.startswith("rel_") for v in case[k]]))
            print(f"[noise] width {width} {mode}: floor max {case['floor_max']:.3e} mean {case['floor_mean']:.3e}",
                  flush=True)
            res["cases"].append(case)
    Path(args.out).write_text(json.dumps(res, indent=1))
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
