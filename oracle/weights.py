"""Deterministic synthetic LLaMA parameters — TEST INFRASTRUCTURE ONLY.

This module belongs to the oracle (see oracle/__init__.py): only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may import it.

No real LLaMA checkpoint is reachable offline, so every parity case is defined by a
seed: the parameters are drawn from numpy's PCG64 stream, which is bit-stable for a
given numpy version, so the golden fixtures (made in the build container by importing
the reference) and the tests (run here and on the GPU box) see identical weights
without shipping them.

Key names follow the reference state_dict contract (reference
lit_llama/model.py:59-72,154-160,178-186,246-255; scripts/convert_checkpoint.py:20-52):
    lm_head.weight, transformer.wte.weight, transformer.ln_f.scale,
    transformer.h.{i}.rms_1.scale, .attn.c_attn.weight, .attn.c_proj.weight,
    .rms_2.scale, .mlp.c_fc1.weight, .mlp.c_fc2.weight, .mlp.c_proj.weight
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def find_multiple(n: int, k: int) -> int:
    """reference lit_llama/utils.py:39-42"""
    if n % k == 0:
        return n
    return n + k - (n % k)


@dataclass
class Cfg:
    """Mirror of reference LLaMAConfig (lit_llama/model.py:23-35)."""

    block_size: int = 2048
    vocab_size: int = 32000
    padded_vocab_size: int | None = None
    n_layer: int = 32
    n_head: int = 32
    n_embd: int = 4096

    def __post_init__(self):
        if self.padded_vocab_size is None:
            self.padded_vocab_size = find_multiple(self.vocab_size, 64)

    @property
    def head_size(self) -> int:
        return self.n_embd // self.n_head

    @property
    def n_hidden(self) -> int:
        # reference lit_llama/model.py:249-251
        return find_multiple(int(2 * (4 * self.n_embd) / 3), 256)


def linear_shapes(cfg: Cfg):
    """(name, out_features, in_features) for every Linear in model order."""
    C, H = cfg.n_embd, cfg.n_hidden
    out = []
    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}."
        out += [
            (p + "attn.c_attn", 3 * C, C),
            (p + "attn.c_proj", C, C),
            (p + "mlp.c_fc1", H, C),
            (p + "mlp.c_fc2", H, C),
            (p + "mlp.c_proj", C, H),
        ]
    out.append(("lm_head", cfg.padded_vocab_size, C))
    return out


def make_params(cfg: Cfg, seed: int, *, wte_std: float = 1.0, lin_gain: float = 1.0,
                head_gain: float = 2.0) -> dict[str, np.ndarray]:
    """fp32 parameters with O(1) activations so greedy top-1/top-2 margins are wide.

    Linear weights ~ N(0, gain/sqrt(in_features)); embedding ~ N(0, wte_std);
    RMSNorm scales ~ U(0.5, 1.5) so the norm weight is exercised non-trivially.
    """
    rng = np.random.default_rng(seed)
    C = cfg.n_embd
    p: dict[str, np.ndarray] = {}
    p["transformer.wte.weight"] = (rng.standard_normal((cfg.padded_vocab_size, C), dtype=np.float32) * wte_std)
    for name, n_out, n_in in linear_shapes(cfg):
        g = head_gain if name == "lm_head" else lin_gain
        p[name + ".weight"] = rng.standard_normal((n_out, n_in), dtype=np.float32) * np.float32(g / np.sqrt(n_in))
    for i in range(cfg.n_layer):
        p[f"transformer.h.{i}.rms_1.scale"] = rng.uniform(0.5, 1.5, C).astype(np.float32)
        p[f"transformer.h.{i}.rms_2.scale"] = rng.uniform(0.5, 1.5, C).astype(np.float32)
    p["transformer.ln_f.scale"] = rng.uniform(0.5, 1.5, C).astype(np.float32)
    return p


def make_prompt(n: int, vocab: int, seed: int, batch: int | None = None) -> np.ndarray:
    rng = np.random.default_rng(seed + 7919)
    shape = (n,) if batch is None else (batch, n)
    return rng.integers(3, vocab, size=shape).astype(np.int32)


def ref_init_params(cfg: Cfg, seed: int) -> dict[str, np.ndarray]:
    """fp32 parameters at the reference's own init scale (lit_llama/model.py:78-82,
    LLaMA._init_weights: every Linear and the Embedding ~ N(0, 0.02 / sqrt(2 * n_layer)); RMSNorm
    scales stay 1, model.py:270), drawn from numpy's PCG64 so a fixture made by the reference
    and a test on the GPU box see identical weights. This is the regime of the reference's bf16
    acceptance test (tests/test_model.py:103-131)."""
    rng = np.random.default_rng(seed)
    std = np.float32(0.02 / np.sqrt(2 * cfg.n_layer))
    C = cfg.n_embd
    p: dict[str, np.ndarray] = {}
    p["transformer.wte.weight"] = rng.standard_normal((cfg.padded_vocab_size, C), dtype=np.float32) * std
    for name, n_out, n_in in linear_shapes(cfg):
        p[name + ".weight"] = rng.standard_normal((n_out, n_in), dtype=np.float32) * std
    for i in range(cfg.n_layer):
        p[f"transformer.h.{i}.rms_1.scale"] = np.ones(C, np.float32)
        p[f"transformer.h.{i}.rms_2.scale"] = np.ones(C, np.float32)
    p["transformer.ln_f.scale"] = np.ones(C, np.float32)
    return p
