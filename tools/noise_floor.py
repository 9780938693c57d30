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
  gpu    (round 4) the base Linears with the decode kernels' own formulas for everything else: RoPE
         as fma(x0, cos, -(x1 sin)) (one rounding), attention scores on q pre-scaled by
         log2(e) / sqrt(hs) with exp2 and the 1 / sum applied after P.V, SiLU as
         x / (1 + exp2(-x log2(e))) -- another valid fp32 evaluation of model.py:237, 258, 312-329.
         Its bf16 flips are what reach LLM.int8's per-row int8 codes (a Linear-order change barely
         moves an int8 model: its GEMM is exact), so it is the variant that prices that mode.

Usage: python tools/noise_floor.py [--out profiles/r04_noise_floor.json] [--batches 1,8]  (CPU, ~10 minutes)
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
        out = out.astype(np.float16).astype(F32)  # mm_dequant's fp16 output (oracle.int8_linear)
        if outl.size:
            wsub = (s.cb[:, outl].astype(F32) * (s.scb[:, None] / F32(127.0))).astype(np.float16).astype(F32)
            out = out + (a16[:, outl].astype(np.float64) @ wsub.T.astype(np.float64)).astype(F32)
        out = out.astype(np.float16).astype(F32)
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


class GpuFormulaOracle(O.OracleLLaMA):
    """The oracle with the decode kernels' formulas for RoPE, softmax and SiLU (Linears as base)."""

    LOG2E = F32(1.4426950408889634)

    @staticmethod
    def _rope(x, rope):
        B, T, nh, hs = x.shape
        xs = x.astype(np.float64).reshape(B, T, nh, hs // 2, 2)
        r = rope[:T].reshape(1, T, 1, hs // 2, 2).astype(np.float64)
        # fma(x0, c, -(x1 s)): the product x1 s rounded to fp32, the rest in one rounding
        t0 = (xs[..., 1] * r[..., 1]).astype(F32).astype(np.float64)
        t1 = (xs[..., 0] * r[..., 1]).astype(F32).astype(np.float64)
        o0 = (xs[..., 0] * r[..., 0] - t0).astype(F32)
        o1 = (xs[..., 1] * r[..., 0] + t1).astype(F32)
        return np.stack([o0, o1], -1).reshape(B, T, nh, hs).astype(F32)

    def _block(self, i, x, rope, mask, S, input_pos):
        cfg, p, pre = self.cfg, self.p, f"transformer.h.{i}."
        B, T, C = x.shape
        nh, hs = cfg.n_head, cfg.head_size
        h = self._norm(x, p[pre + "rms_1.scale"])
        qkv = self._r(self.lin[pre + "attn.c_attn"](h))
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        q = self._r(self._rope(q.reshape(B, T, nh, hs), rope)).transpose(0, 2, 1, 3)
        k = self._r(self._rope(k.reshape(B, T, nh, hs), rope)).transpose(0, 2, 1, 3)
        v = v.reshape(B, T, nh, hs).transpose(0, 2, 1, 3)
        if input_pos is not None:
            ck, cv = self.kv[i]
            pos = input_pos
            if pos[-1] >= S:
                pos = np.array([S - 1])
                ck = np.roll(ck, -1, axis=2)
                cv = np.roll(cv, -1, axis=2)
            ck = ck.copy(); cv = cv.copy()
            ck[:, :, pos] = k
            cv[:, :, pos] = v
            self.kv[i] = [ck, cv]
            k, v = ck, cv
        qs = (q * (self.LOG2E / F32(np.sqrt(F32(hs))))).astype(F32)
        att = (qs @ k.transpose(0, 1, 3, 2)).astype(F32)
        att = np.where(mask[None, None], att, -np.inf)
        e = np.exp2((att - att.max(-1, keepdims=True)).astype(F32)).astype(F32)
        y = ((e @ v).astype(F32) / e.sum(-1, keepdims=True, dtype=F32)).astype(F32)
        y = self._r(y.transpose(0, 2, 1, 3).reshape(B, T, C))
        x = self._r(x + self._r(self.lin[pre + "attn.c_proj"](y)))
        h = self._norm(x, p[pre + "rms_2.scale"])
        a1 = self._r(self.lin[pre + "mlp.c_fc1"](h))
        a2 = self._r(self.lin[pre + "mlp.c_fc2"](h))
        sl = (a1 / (F32(1.0) + np.exp2((-a1 * self.LOG2E).astype(F32)))).astype(F32)
        m = self._r(self._r(sl) * a2)
        return self._r(x + self._r(self.lin[pre + "mlp.c_proj"](m)))


def orc_variant(cfg, pb, lin, order):
    if order == "base":
        return O.OracleLLaMA(cfg, pb, linears=lin, act_bf16=True)
    if order == "gpu":
        return GpuFormulaOracle(cfg, pb, linears=lin, act_bf16=True)
    return AltOracle(cfg, pb, lin, order)


ORDERS = ("base", "f64", "chunk", "gpu")


def pair_rels(outs):
    """rel L2 of every pair of variants, per (row, step)"""
    keys = list(outs)
    return {f"rel_{a}_vs_{b}": rels(outs[a], outs[b]) for i, a in enumerate(keys) for b in keys[i + 1:]}


def rels(a, b):
    return [float(np.linalg.norm(a[i, s] - b[i, s]) / np.linalg.norm(b[i, s]))
            for i in range(a.shape[0]) for s in range(a.shape[1])]


def _case(name, outs):
    case = {"case": name, **pair_rels(outs)}
    case["floor_max"] = max(max(case[k]) for k in case if k.startswith("rel_"))
    case["floor_mean"] = float(np.mean([v for k in case if k.startswith("rel_") for v in case[k]]))
    print(f"[noise] {name}: floor max {case['floor_max']:.3e} mean {case['floor_mean']:.3e}", flush=True)
    return case


def generic_cases(generic_modes=(None, "gptq.int4", "llm.int8")):
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
    for mode in generic_modes:
        pb, _, lin = T.oracle_linears(p, mode)
        outs_rows, outs_steps = {}, {}
        for o in ("base", "f64", "chunk", "gpu"):
            st, rows = T._oracle_steps(orc_variant(cfg, pb, lin, o), ids, t_prompt=12, steps=4, s=32, all_rows=True)
            outs_rows[o], outs_steps[o] = rows, st
        cases.append(_case(f"125M {mode} prompt rows", outs_rows))
        cases.append(_case(f"125M {mode} steps", outs_steps))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--widths", default="4096,5120")
    ap.add_argument("--batches", default="1,8")
    ap.add_argument("--modes", default=None, help="comma list of gptq.int4, bf16, llm.int8 (default: all)")
    ap.add_argument("--generic", action="store_true")
    ap.add_argument("--prefill", action="store_true")
    args = ap.parse_args()
    res = {"what": __doc__.split("\n\n")[0], "cases": []}
    if args.generic:
        gm = (None, "gptq.int4", "llm.int8") if not args.modes else tuple(
            None if m == "bf16" else m for m in args.modes.split(","))
        res["cases"] = generic_cases(gm)
        out = args.out or str(REPO / "profiles" / "r04_noise_floor_generic.json")
        Path(out).write_text(json.dumps(res, indent=1))
        print(f"wrote {out}")
        return
    if args.prefill:  # the 64-token prompt tests (test_7b_width_prefill_gemm_flash_vs_oracle, 13B likewise)
        for width in [int(w) for w in args.widths.split(",")]:
            cfg = T.C7 if width == 4096 else T.C13
            p = T.make_params(cfg, T.SEEDS[width])
            modes = ["gptq.int4", None, "llm.int8"] if width == 4096 else ["gptq.int4"]
            if args.modes:
                modes = [None if m == "bf16" else m for m in args.modes.split(",")
                         if (m == "bf16" and None in modes) or m in modes]
            for mode in modes:
                pb, _, lin = T.oracle_linears(p, mode)
                ids = np.random.default_rng(64 if width == 4096 else 65).integers(3, cfg.vocab_size, (1, 64 + 3))
                rows, steps = {}, {}
                for order in ORDERS:
                    t0 = time.time()
                    steps[order], rows[order] = T._oracle_steps(orc_variant(cfg, pb, lin, order), ids, t_prompt=64,
                                                                steps=2, s=96, all_rows=True)
                    print(f"[noise] prefill width {width} {mode} {order}: {time.time() - t0:.1f} s", flush=True)
                res["cases"].append(_case(f"prefill 64 rows width {width} {mode}", rows))
                res["cases"].append(_case(f"prefill steps width {width} {mode}", steps))
        out = args.out or str(REPO / "profiles" / "r04_noise_floor_prefill.json")
        Path(out).write_text(json.dumps(res, indent=1))
        print(f"wrote {out}")
        return
    args.out = args.out or str(REPO / "profiles" / "r04_noise_floor.json")
    batches = [int(b) for b in args.batches.split(",")]
    for width in [int(w) for w in args.widths.split(",")]:
        cfg = T.C7 if width == 4096 else T.C13
        p = T.make_params(cfg, T.SEEDS[width])
        modes = ["gptq.int4", None, "llm.int8"] if width == 4096 else ["gptq.int4"]
        if args.modes:
            modes = [None if m == "bf16" else m for m in args.modes.split(",") if (m == "bf16" and None in modes) or m in modes]
        for mode in modes:
            pb, _, lin = T.oracle_linears(p, mode)
            for B in batches:
                rng_seed = (B + 17) if width == 4096 else (B + 31)  # the tests' ids for this batch
                ids = np.random.default_rng(rng_seed).integers(3, cfg.vocab_size, (B, T.T_PROMPT + T.STEPS + 1))
                outs = {}
                for order in ORDERS:
                    t0 = time.time()
                    outs[order] = T._oracle_steps(orc_variant(cfg, pb, lin, order), ids)
                    print(f"[noise] width {width} {mode} B={B} {order}: {time.time() - t0:.1f} s", flush=True)
                case = {"width": width, "mode": str(mode), "batch": B, "steps": T.STEPS + 1, **pair_rels(outs)}
                allr = [v for k in case if k.startswith("rel_") for v in case[k]]
                case["floor_max"] = max(allr)
                case["floor_mean"] = float(np.mean(allr))
                gpu = [v for k in case if k.startswith("rel_") and "gpu" in k for v in case[k]]
                case["floor_max_gpu_formulas"] = max(gpu)
                print(f"[noise] width {width} {mode} B={B}: floor max {case['floor_max']:.3e} mean "
                      f"{case['floor_mean']:.3e} (gpu-formula pairs max {case['floor_max_gpu_formulas']:.3e})", flush=True)
                res["cases"].append(case)
    Path(args.out).write_text(json.dumps(res, indent=1))
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
