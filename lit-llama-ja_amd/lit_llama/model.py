"""LLaMA for the MI355X decode path: the reference's module tree and API (lit_llama/model.py),
with LLaMA.forward executed by the fused gfx950 kernels of _lljamd.so.

Same as the reference (if001/lit-llama-ja lit_llama/model.py): LLaMAConfig + llama_configs
(23-56), parameter/buffer names and shapes (state_dict compatible), LLaMA.forward(idx,
max_seq_length, input_pos) -> logits (59-128), lazily allocated per-layer KV caches
(115-121), reset_cache, from_name, build_rope_cache / build_mask_cache, RMSNorm, apply_rope.

Execution per Block (model.py:162-175) is four weight-streaming launches plus attention:
  1. rms_1 + c_attn + RoPE(q, k) + KV write        (llj_norm_qkv_rope)
  2. causal attention over the cache              (llj_attention)
  3. c_proj + residual add                         (llj_linear_resid)
  4. rms_2 + c_fc1 / c_fc2 + silu * mul            (llj_norm_swiglu)
  5. mlp.c_proj + residual add                     (llj_linear_resid)
and ln_f + lm_head (llj_norm_linear). The KV cache is a ring: the token at absolute
position p is stored in slot p % S, which holds the same key set as the reference's
roll-by-one sliding window (model.py:221-227); `kv_caches` therefore equals the reference's
caches up to a rotation of the slot axis once more than S tokens were seen.

The model must live on a ROCm GPU, in bfloat16 (the reference's GPU precision, generate.py:121) or
in float32 (the reference's CPU / evaluate/full.py default precision: every op then runs on the
any-shape kernels in fp32); there is no CPU path.
"""
from __future__ import annotations

import math
import os
import types
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
from typing_extensions import Self

from . import _hip
from .utils import find_multiple

MaskCache = torch.Tensor
RoPECache = torch.Tensor
KVCache = Tuple[torch.Tensor, torch.Tensor]


@dataclass
class LLaMAConfig:
    block_size: int = 2048
    vocab_size: int = 32000
    padded_vocab_size: Optional[int] = None
    n_layer: int = 32
    n_head: int = 32
    n_embd: int = 4096

    def __post_init__(self):
        if self.padded_vocab_size is None:
            self.padded_vocab_size = find_multiple(self.vocab_size, 64)

    @classmethod
    def from_name(cls, name: str) -> Self:
        return cls(**llama_configs[name])

    def kernel_support(self) -> Optional[str]:
        """None if the streaming gfx950 kernels take this configuration, else why not -- such a
        model runs on the any-shape kernels (csrc/generic.hip) instead. The GEMVs stream 128-deep
        K chunks and 16-column tiles (n_embd % 128 == 0; n_hidden, 3 n_embd and the padded vocab
        are then multiples of 16), the fused RoPE / attention kernels take head_size 64 or 128. The
        JA fork's 19M / 49M configs (head 64), 7B / 13B / 30B / 65B (head 128) take the streaming
        path; its 125M config (n_embd 780, head 78) and the reference test's n_embd 32 / head 2 the
        any-shape path."""
        hs = self.n_embd // self.n_head
        if self.n_embd % self.n_head:
            return f"n_embd {self.n_embd} is not a multiple of n_head {self.n_head}"
        if self.n_embd % 128:
            return f"n_embd {self.n_embd} is not a multiple of 128 (the GEMV K chunk)"
        if hs not in (64, 128):
            return f"head_size {hs} is not 64 or 128 (fused RoPE / attention kernels)"
        return None

    def debug(self):
        for k in ("block_size", "vocab_size", "padded_vocab_size", "n_layer", "n_head", "n_embd"):
            print(f"{k}: ", getattr(self, k))


llama_configs = {
    "19M": dict(n_layer=6, n_head=8, n_embd=512, vocab_size=35000),
    "49M": dict(n_layer=10, n_head=10, n_embd=640, vocab_size=35000),
    "125M": dict(n_layer=12, n_head=10, n_embd=780, vocab_size=35000),
    "7B": dict(n_layer=32, n_head=32, n_embd=4096),
    "13B": dict(n_layer=40, n_head=40, n_embd=5120),
    "30B": dict(n_layer=60, n_head=52, n_embd=6656),
    "65B": dict(n_layer=80, n_head=64, n_embd=8192),
}

QKV_ROWS = 8    # fused-norm kernels stage <= 8 rows in LDS
LIN_ROWS = 16   # plain linear kernels take <= 16 rows per launch
I8_ROWS = 8     # int8 kernels quantize <= 8 rows in LDS
if os.environ.get("LLJ_I8_ROWS"):  # profiling only: smaller int8 row slices (A images under 64 KiB of LDS)
    I8_ROWS = max(1, min(8, int(os.environ["LLJ_I8_ROWS"])))
# long caches: attention split over the keys (llj_attention_split) into ATTN_SPLIT_KEYS-key
# ranges once the cache holds >= ATTN_SPLIT_MIN_S slots (32 heads x 1 row leave most CUs idle)
ATTN_SPLIT_MIN_S = 512
ATTN_SPLIT_KEYS = 256  # 7B bs=1 at p = 2000 (S = 2048): 33.1 us one block, 14.4 us in 8 ranges


# prompts of at least this many tokens run the MFMA flash attention (llj_attention_prefill) when
# their positions are contiguous and do not wrap the ring
FLASH_MIN_T = 32


# decode attention of ONE row as ATT_MERGE interleaved key splits per head (llj_attention_part) merged in
# attn.c_proj's prologue (llj_linear_resid_attn) instead of one block per head; 0 = off (A/B, verdict r5 #4)
ATT_MERGE = 0


def attn_splits(S: int) -> int:
    """key ranges per (row, head) for a cache of S slots (1 = the one-block attention)."""
    if S < ATTN_SPLIT_MIN_S:
        return 1
    return min(64, (S + ATTN_SPLIT_KEYS - 1) // ATTN_SPLIT_KEYS)
# batched rows (M >= 2): each RMSNorm as its own launch (llj_rmsnorm_rows) feeding LDS-A GEMVs,
# instead of normalized inside every norm-fused GEMV workgroup
PRE_NORM_ROWS = True
PRE_NORM_MIN_M = 2  # smallest batch that takes the separate launch (measured best from bs=2 on)
# batched decode rows (2 <= M <= HAND_NORM_MAX_M): the residual ops hand the next RMSNorm its sums
# of squares (per-tile partials, llj_linear_resid's nstat_out) and the norm-fused GEMVs normalize
# from them, so no separate RMSNorm launch remains after layer 0's rms_1. With the LDS-image GEMVs
# (round 3, every workgroup normalizing all rows before its stream) this lost from bs=3 on (7B
# gptq.int4 ms/token, hand-off vs llj_rmsnorm_rows: bs=4 1.633 vs 1.539, bs=8 1.877 vs 1.788); the
# streamed-A GEMVs (gemv_impl.h AM_SNORM) normalize each chunk's rows as they arrive, so every batch
# up to 8 rows takes the hand-off
HAND_NORM = True
HAND_NORM_MAX_M = 8
HAND_NORM_MIN_M = 2  # 1: single rows too (with llj_set_stream_a(2); A/B)


# prefill / no-cache calls with at least this many rows (B * T) run the MFMA-tiled GEMMs
# (llj_gemm_*) instead of the weight-streaming GEMVs in 8 / 16-row slices, when every Linear of
# the model is int4 W4P (per-row or grouped scales), gptq.int8 W8P, LLM.int8 I8P (int8 MFMA + fp16
# outlier side product, llj_gemm_i8_*) or bf16 and the shapes tile by 128
GEMM_MIN_ROWS = 32
_GEMM_FMTS = (0, 1, 2, 3, 4)  # weight formats (low byte of wfmt; 4 = grouped int4) the prefill GEMMs take


def _gemm_fmt(wfmt: int) -> bool:
    return (wfmt & 0xFF) in _GEMM_FMTS


# int4 prompt GEMMs of Linears whose zeros are all integers (GPTQ's round(-min / scale)): each chunk's
# codes converted once per workgroup into an exact bf16 (q - z) tile, the scale in the epilogue
# (LLJ_WF_ZINT; csrc/gemm.hip, the convert-once LDS-DMA kernel at M >= 256)
GEMM_ZINT = True
# ... and c_fc1 / c_fc2 of such weights in one dual pass (llj_gemm_swiglu: one A tile for both, silu * mul
# in the epilogue, no h round trip) at M >= 256
GEMM_SWIGLU = True


def _gz(wfmt: int, lin: nn.Module) -> int:
    """wfmt of a prompt-GEMM call on `lin`: int4 with LLJ_WF_ZINT when its zeros are integers."""
    if GEMM_ZINT and wfmt == 0 and hasattr(lin, "zeros_integral") and lin.zeros_integral():
        return wfmt | _hip.WF_ZINT
    return wfmt

# LLM.int8 prompt rows: the outlier columns of each GEMM's activation and weight pre-gathered as f16
# rows (llj_i8_gather_act / _weight), so the fp16 side product runs as a dense f16 GEMM over them
I8_GATHER = True
# their capacity in outlier columns: all of K while the f16 weight rows of one call stay within
# I8_GATHER_BUDGET bytes (7B: every Linear; the 65B c_fc1 + c_fc2 pair caps at 2,880 columns), and
# at most I8_GATHER_MAX, the gathers' LDS list ((80 + kpad) * 4 <= 64 KiB); real checkpoints have
# 6-20 outlier columns, synthetic random weights up to all of K
I8_GATHER_BUDGET = 256 << 20
I8_GATHER_MAX = 16256

# int8 decode: RMSNorm + LLM.int8() statistics in one launch pair up to this many rows
I8_NORM_STATS_MAX_M = 16
# int8 decode rows (M <= I8S_MAX_M): the attention output's and the SwiGLU output's LLM.int8
# statistics come from the ops that produce them (llj_attention_i8, llj_i8_swiglu_stats) and the
# int8 c_proj / mlp.c_proj quantize their rows per chunk (llj_i8_linear_resid): no statistics launch
# for y and h
I8_HANDOFF = True
I8S_MAX_M = 8
# ... and the norm outputs (rms_1 / rms_2 / ln_f rows) quantized per chunk inside the int8 GEMVs from a
# hand-off block written by their statistics launch (llj_i8_norm_rowstats), instead of the launch's
# quantized rows staged in LDS: measured slower (7B llm.int8 bs=8: QKV 14.8 -> 19.1 us, C3 2,671 ->
# 2,436 tokens/s; the 768 / 688 workgroups re-quantize the same rows), so off
I8_NORM_ROWSTATS = False

# weight formats whose kernels remove the nibble offset with the row sums of A (W4P, W8P)
_ROWSUM_FMTS = (0, 3)


def _dt_code(dtype) -> int:
    """dt argument of the any-shape kernels: 0 bf16, 1 fp32."""
    if dtype == torch.bfloat16:
        return 0
    if dtype == torch.float32:
        return 1
    raise TypeError(f"activations must be bfloat16 or float32, got {dtype}")


def _wspec(lin: nn.Module):
    """(wfmt, weight operand, scale operand) of a Linear for the HIP kernels."""
    if hasattr(lin, "_wspec"):
        return lin._wspec()
    if isinstance(lin, nn.Linear):
        w = lin.weight
        _hip.require_device(w, "Linear.weight")
        if w.dtype != torch.bfloat16 or not w.is_contiguous():
            raise TypeError("dense Linear weights must be contiguous bfloat16 on the GPU "
                            "(construct under EmptyInitOnDevice(dtype=torch.bfloat16) or call .to(torch.bfloat16))")
        if lin.bias is not None:
            raise NotImplementedError("biased dense Linear is not on the LLaMA path")
        return 1, w, None
    raise TypeError(f"unsupported Linear class {type(lin).__name__}")


def _gspec(lin: nn.Module):
    """Operands of a Linear for the any-shape kernel llj_g_linear: (wkind, W, scales, zeros, bits,
    group) -- wkind 1 dense (bf16 or fp32, the activation type), 0 ColBlockQuantizedLinear on its
    reference buffers."""
    if hasattr(lin, "_gspec"):
        return lin._gspec()
    if isinstance(lin, nn.Linear):
        w = lin.weight
        _hip.require_device(w, "Linear.weight")
        if w.dtype not in (torch.bfloat16, torch.float32) or not w.is_contiguous():
            raise TypeError("dense Linear weights must be contiguous bfloat16 or float32 on the GPU")
        if lin.bias is not None:
            raise NotImplementedError("biased dense Linear is not on the LLaMA path")
        return 1, w, None, None, 16, w.shape[1]
    raise NotImplementedError(f"{type(lin).__name__} has no any-shape kernel")


def _enable_i8_handoff(w: "_Work", specs) -> None:
    """The LLM.int8 statistics hand-off (see _Work) when every Linear of every layer is LLM.int8."""
    w.i8s = w.y_st is not None and all(s[0] == 2 for layer in specs["layers"] for s in layer)


class _Work:
    """Per-call scratch for M rows (allocated from torch's caching allocator)."""

    def __init__(self, cfg: LLaMAConfig, M: int, device, need_i8: bool, S: int = 0, gemm: bool = False,
                 generic: bool = False, dtype=torch.bfloat16):
        C, H = cfg.n_embd, MLP.hidden(cfg)
        bf = torch.bfloat16
        self.generic = generic  # the any-shape kernels (LLaMA._blocks_generic)
        self.dt = _dt_code(dtype)
        if generic:
            bf = dtype  # fp32 models run here with fp32 activations
            self.x = torch.empty(M, C, dtype=bf, device=device)
            self.xn = torch.empty(M, C, dtype=bf, device=device)
            self.qkv = torch.empty(M, 3 * C, dtype=bf, device=device)
            self.q = torch.empty(M, C, dtype=bf, device=device)
            self.y = torch.empty(M, C, dtype=bf, device=device)
            self.a1 = torch.empty(M, H, dtype=bf, device=device)
            self.a2 = torch.empty(M, H, dtype=bf, device=device)
            self.h = torch.empty(M, H, dtype=bf, device=device)
            self.gemm = self.flash = self.pre = self.hand = False
            self.i8ws = self.att_ws = self.nst = self.rs = None
            return
        self.gemm = gemm  # many rows: the prefill GEMMs (LLaMA._blocks_gemm)
        self.flash = False  # T-row prompt attention on the MFMA flash kernel (set by LLaMA._run)
        self.x = torch.empty(M, C, dtype=bf, device=device)
        self.q = torch.empty(M, C, dtype=bf, device=device)
        self.y = torch.empty(M, C, dtype=bf, device=device)
        self.h = torch.empty(M, H, dtype=bf, device=device)
        # batched rows (M >= 2): each RMSNorm runs once (llj_rmsnorm_rows -> xn, rs = fp32 row
        # sums for the int4 offset term) instead of inside every norm-fused GEMV workgroup
        self.pre = M >= max(2, PRE_NORM_MIN_M) and not need_i8 and PRE_NORM_ROWS
        self.xn = torch.empty(M, C, dtype=bf, device=device) if (need_i8 or self.pre or gemm) else None
        self.rs = torch.empty(M, dtype=torch.float32, device=device) if self.pre else None
        # norm statistics hand-off (HAND_NORM): partials [C / 16 tiles][16 rows]
        self.hand = (HAND_NORM and not need_i8 and not gemm and HAND_NORM_MIN_M <= M <= HAND_NORM_MAX_M
                     and C % 16 == 0 and C // 16 <= 512)
        self.npart = C // 16
        self.nst = torch.empty(self.npart * 16, dtype=torch.float32, device=device) if self.hand else None
        if need_i8:
            L = _hip.lib()
            nb = max(L.llj_i8_ws_bytes(M, C), L.llj_i8_ws_bytes(M, H))
            self.i8ws = torch.empty(nb, dtype=torch.uint8, device=device)
        else:
            self.i8ws = None
        # LLM.int8 decode rows (M <= 8, every Linear int8; enable_i8_handoff): the attention and the
        # int8 SwiGLU hand their outputs' LLM.int8 statistics to the int8 c_proj / mlp.c_proj (i8ws.h
        # kI8StFlags blocks, zero at allocation; a step leaves y's zero again)
        self.i8s = False
        self.y_st = self.h_st = self.n_st = None
        if need_i8 and not gemm and M <= I8S_MAX_M and I8_HANDOFF:
            L = _hip.lib()
            self.y_st = torch.zeros(L.llj_i8_rowstats_bytes(C) // 4, dtype=torch.int32, device=device)
            self.h_st = torch.zeros(L.llj_i8_rowstats_bytes(H) // 4, dtype=torch.int32, device=device)
            # the norm outputs' block (rms_1 / rms_2 / ln_f), rewritten whole by llj_i8_norm_rowstats
            self.n_st = torch.zeros(L.llj_i8_rowstats_bytes(C) // 4, dtype=torch.int32, device=device)
        # split-K attention partials for long caches (llj_attention_split)
        self.nsplit = attn_splits(S)
        self.att_ws = None
        if self.nsplit > 1:
            nb = _hip.lib().llj_attention_ws_bytes(M, cfg.n_head, C // cfg.n_head, self.nsplit)
            self.att_ws = torch.empty(nb, dtype=torch.uint8, device=device)
        # one decode row, short cache: interleaved split partials merged in attn.c_proj (ATT_MERGE)
        self.att_merge = ATT_MERGE if (ATT_MERGE > 1 and M == 1 and self.nsplit <= 1 and not need_i8) else 0
        self.att_part = None
        if self.att_merge:
            nb = _hip.lib().llj_attention_ws_bytes(1, cfg.n_head, C // cfg.n_head, self.att_merge)
            self.att_part = torch.empty(nb, dtype=torch.uint8, device=device)


class LLaMA(nn.Module):
    def __init__(self, config: LLaMAConfig) -> None:
        super().__init__()
        assert config.padded_vocab_size is not None
        self.config = config
        self.lm_head = nn.Linear(config.n_embd, config.padded_vocab_size, bias=False)
        self.transformer = nn.ModuleDict(
            dict(
                wte=nn.Embedding(config.padded_vocab_size, config.n_embd),
                h=nn.ModuleList(Block(config) for _ in range(config.n_layer)),
                ln_f=RMSNorm(config.n_embd),
            )
        )
        self.rope_cache: Optional[RoPECache] = None
        self.mask_cache: Optional[MaskCache] = None
        self.kv_caches: List[KVCache] = []

    def _init_weights(self, module: nn.Module) -> None:
        """reference model.py:78-82"""
        if isinstance(module, nn.Linear):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02 / math.sqrt(2 * self.config.n_layer))
        elif isinstance(module, nn.Embedding):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02 / math.sqrt(2 * self.config.n_layer))

    @classmethod
    def from_name(cls, name: str) -> Self:
        return cls(LLaMAConfig.from_name(name))

    def build_rope_cache(self, idx: torch.Tensor) -> RoPECache:
        return build_rope_cache(seq_len=self.config.block_size, n_elem=self.config.n_embd // self.config.n_head,
                                dtype=idx.dtype, device=idx.device)

    def build_mask_cache(self, idx: torch.Tensor) -> MaskCache:
        ones = torch.ones((self.config.block_size, self.config.block_size), device=idx.device, dtype=torch.bool)
        return torch.tril(ones).unsqueeze(0).unsqueeze(0)

    def reset_cache(self) -> None:
        """reference model.py:146-151"""
        self.kv_caches.clear()

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, idx: torch.Tensor, max_seq_length: Optional[int] = None,
                input_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, T = idx.size()
        block_size = self.config.block_size
        if max_seq_length is None:
            max_seq_length = block_size
        assert T <= max_seq_length, f"Cannot forward sequence of length {T}, max seq length is only {max_seq_length}"
        assert max_seq_length <= block_size, f"Cannot attend to {max_seq_length}, block size is only {block_size}"
        assert T <= block_size, f"Cannot forward sequence of length {T}, block size is only {block_size}"
        _hip.require_device(idx, "idx")
        self._check_dtype()
        if self.rope_cache is None:
            self.rope_cache = self.build_rope_cache(idx)
        if input_pos is None:
            # no-cache path (model.py:111-113): causal attention over the T tokens themselves,
            # i.e. fresh caches of length T written at positions 0..T-1
            pos = torch.arange(T, device=idx.device, dtype=torch.int32)
            kv = self._alloc_kv(B, T, idx.device, n=1)
            kv = kv * self.config.n_layer
            return self._run(idx, pos, T, kv, all_rows=True)
        pos = input_pos.to(device=idx.device, dtype=torch.int32)
        assert pos.numel() == T, "input_pos must have one position per token"
        if not self.kv_caches:
            self.kv_caches = self._alloc_kv(B, max_seq_length, idx.device)
        S = self.kv_caches[0][0].shape[2]
        if S != max_seq_length or self.kv_caches[0][0].shape[0] != B:
            raise ValueError(f"KV cache was allocated for batch {self.kv_caches[0][0].shape[0]} and "
                             f"max_seq_length {S}; call reset_cache() first")
        return self._run(idx, pos, S, self.kv_caches, all_rows=True)

    def _alloc_kv(self, B, S, device, n=None):
        hs = self.config.n_embd // self.config.n_head
        shape = (B, self.config.n_head, S, hs)
        dt = self.act_dtype()  # the reference's cache dtype is the activation dtype (model.py:117-120)
        return [(torch.zeros(shape, device=device, dtype=dt), torch.zeros(shape, device=device, dtype=dt))
                for _ in range(self.config.n_layer if n is None else n)]

    def act_dtype(self) -> torch.dtype:
        """The activation dtype: the embedding's (bf16 or fp32)."""
        return self.transformer.wte.weight.dtype

    def _check_dtype(self):
        wte = self.transformer.wte.weight
        _hip.require_device(wte, "LLaMA parameters")
        if wte.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError("the MI355X path computes in bfloat16 or float32: build the model under "
                            "EmptyInitOnDevice(device='cuda', dtype=torch.bfloat16) or call model.to(torch.bfloat16)")
        if wte.dtype == torch.float32:  # the fp32 model: every norm / dense weight fp32 as well
            for n, prm in self.named_parameters():  # (LLM.int8's CB is int8 under any activation dtype)
                if prm.dtype != torch.float32 and not (prm.dtype == torch.int8 and n.endswith(".weight")):
                    raise TypeError(f"float32 model with a {prm.dtype} parameter {n}")

    def _run(self, idx, pos, S, kv, all_rows=True, last_only_out=None):
        """Embedding -> n_layer blocks -> ln_f -> lm_head for B*T rows; returns (B, T, V)
        logits (or only the last position of each sequence into `last_only_out` (B, V))."""
        cfg = self.config
        B, T = idx.shape
        M = B * T
        dev = idx.device
        specs = self._layer_specs()
        if self._generic():
            w = _Work(cfg, M, dev, False, S, generic=True, dtype=self.act_dtype())
        else:
            need_i8 = any(s[0] == 2 for layer in specs["layers"] for s in layer) or specs["head"][0] == 2
            w = _Work(cfg, M, dev, need_i8, S, gemm=self._gemm_ok(specs, M))
            w.flash = self._flash_ok(pos, T, S)
            _enable_i8_handoff(w, specs)
        st = _hip.stream()
        ids = idx.reshape(-1).to(torch.int32)
        if w.generic:
            _hip.call("llj_g_embedding", ids.data_ptr(), self.transformer.wte.weight.data_ptr(), w.x.data_ptr(), M,
                      cfg.n_embd, None, w.dt, st)
        else:
            _hip.call("llj_embedding", ids.data_ptr(), self.transformer.wte.weight.data_ptr(), w.x.data_ptr(), M,
                      cfg.n_embd, None, st)
        self._blocks(w, specs, kv, pos, B, T, S, st)
        V = cfg.padded_vocab_size
        if last_only_out is not None:
            if T == 1:
                self._head(w.x, B, specs, last_only_out, st, w)
            else:
                rows = w.x.view(B, T, -1)[:, -1].contiguous()
                self._head(rows, B, specs, last_only_out, st, w)
            return last_only_out
        logits = torch.empty(M, V, dtype=self.act_dtype(), device=dev)
        self._head(w.x, M, specs, logits, st, w)
        return logits.view(B, T, V)

    def _generic(self) -> bool:
        """True when this model runs on the any-shape kernels: a configuration outside the
        streaming tiling (kernel_support), or fp32 activations."""
        return self.config.kernel_support() is not None or self.act_dtype() == torch.float32

    # -- weight operands, gathered once per call
    def _layer_specs(self):
        if self._generic():
            return {"layers": [tuple(_gspec(m) for m in (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc1,
                                                         blk.mlp.c_fc2, blk.mlp.c_proj))
                               for blk in self.transformer.h],
                    "head": _gspec(self.lm_head)}
        layers = []
        for blk in self.transformer.h:
            layers.append((_wspec(blk.attn.c_attn), _wspec(blk.attn.c_proj), _wspec(blk.mlp.c_fc1),
                           _wspec(blk.mlp.c_fc2), _wspec(blk.mlp.c_proj)))
        return {"layers": layers, "head": _wspec(self.lm_head)}

    def _i8_prep(self, A, M, K, w, st):
        _hip.call("llj_i8_stats", A.data_ptr(), A.stride(0), M, K, Linear8bitLtThreshold, w.i8ws.data_ptr(), st)

    def _i8_norm_prep(self, x, norm, xn, M, K, w, st):
        """RMSNorm of x into xn + the int8 statistics of xn: one fused launch pair for decode rows
        (llj_i8_norm_stats, M <= 16), else llj_rmsnorm then llj_i8_stats."""
        if M <= I8_NORM_STATS_MAX_M and x.stride(0) == K:  # (the library falls back by itself past its envelope)
            _hip.call("llj_i8_norm_stats", x.data_ptr(), norm.scale.data_ptr(), norm.eps, xn.data_ptr(), M, K,
                      Linear8bitLtThreshold, w.i8ws.data_ptr(), st)
            return
        _hip.call("llj_rmsnorm", x.data_ptr(), norm.scale.data_ptr(), norm.eps, xn.data_ptr(), M, K, st)
        self._i8_prep(xn, M, K, w, st)

    def _i8_gathered(self, A, M, K, lins, w, st):
        """(ao16, [w16 per (W, sz, N) in lins], kpad): the outlier columns of A (statistics already in
        w.i8ws) and of each weight as f16 rows for the LLM.int8 GEMMs (I8_GATHER), else (None, Nones, 0).
        kpad is a fixed capacity (the count stays on the device): every outlier column while the f16
        weight rows fit I8_GATHER_BUDGET bytes, and at most I8_GATHER_MAX (the gathers' LDS list); a
        count above it gathers nothing and the GEMM runs its per-tile side product.
        Stream-ordered: freed after the call, reused only by later work on the same stream."""
        if not I8_GATHER:
            return None, [None] * len(lins), 0
        rows = sum(N for _, _, N in lins)
        kpad = min((K + 63) // 64 * 64, I8_GATHER_MAX, max(64, I8_GATHER_BUDGET // (2 * rows) // 64 * 64))
        ao = torch.empty(M, kpad, dtype=torch.float16, device=A.device)
        _hip.call("llj_i8_gather_act", A.data_ptr(), A.stride(0), M, K, w.i8ws.data_ptr(), ao.data_ptr(), kpad, st)
        out = []
        for W, sz, N in lins:
            t = torch.empty(N, kpad, dtype=torch.float16, device=A.device)
            _hip.call("llj_i8_gather_weight", W.data_ptr(), _hip.ptr(sz), N, K, w.i8ws.data_ptr(), t.data_ptr(), kpad,
                      st)
            out.append(t)
        return ao, out, kpad

    def _flash_ok(self, pos, T, S):
        """prompt rows attend through the flash kernel: T >= FLASH_MIN_T, head_size 64 / 128,
        positions contiguous and inside the cache without wrapping (one host read of pos; prompts
        only, never inside a captured decode step)."""
        hs = self.config.n_embd // self.config.n_head
        if T < FLASH_MIN_T or hs not in (64, 128):
            return False
        p = pos.cpu()
        return bool((p[1:] - p[:-1] == 1).all()) and int(p[0]) + T <= S

    def _attention(self, w, kc, vc, pos, B, T, S, st):
        cfg = self.config
        C, nh = cfg.n_embd, cfg.n_head
        if w.flash:
            _hip.call("llj_attention_prefill", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), w.y.data_ptr(),
                      pos.data_ptr(), B, T, nh, C // nh, S, st)
        elif w.att_ws is not None:
            _hip.call("llj_attention_split", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), w.y.data_ptr(),
                      pos.data_ptr(), B, T, nh, C // nh, S, w.nsplit, w.att_ws.data_ptr(), st)
        else:
            _hip.call("llj_attention", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), w.y.data_ptr(),
                      pos.data_ptr(), B, T, nh, C // nh, S, st)

    def _gemm_ok(self, specs, M):
        cfg = self.config
        C, H = cfg.n_embd, MLP.hidden(cfg)
        fmts = {s[0] for layer in specs["layers"] for s in layer}
        return (M >= GEMM_MIN_ROWS and all(_gemm_fmt(f) for f in fmts) and C % 128 == 0 and H % 128 == 0
                and _gemm_fmt(specs["head"][0]))

    def _blocks_gemm(self, w, specs, kv, pos, B, T, S, st):
        """The n_layer blocks for many rows through the prefill GEMMs (csrc/gemm.hip): per layer
        rms_1 (llj_rmsnorm_rows) -> c_attn + RoPE + KV write -> attention -> c_proj + residual ->
        rms_2 -> c_fc1, then c_fc2 with the silu * mul epilogue -> mlp.c_proj + residual."""
        cfg = self.config
        C, H, nh = cfg.n_embd, MLP.hidden(cfg), cfg.n_head
        M = B * T
        P = _hip.ptr
        I8ws = P(w.i8ws)
        for i, blk in enumerate(self.transformer.h):
            (fa, wa, sa), (fp, wp, sp), (f1, w1, s1), (f2, w2, s2), (fd, wd, sd) = specs["layers"][i]
            kc, vc = kv[i]
            if fa == 2:  # LLM.int8: the norm + the activation statistics of all M rows, then the int8 GEMM
                self._i8_norm_prep(w.x, blk.rms_1, w.xn, M, C, w, st)
                ao, (wg,), kp = self._i8_gathered(w.xn, M, C, [(wa, sa, 3 * C)], w, st)
                _hip.call("llj_gemm_i8_qkv_rope", w.xn.data_ptr(), wa.data_ptr(), P(sa), I8ws, P(ao), P(wg), kp,
                          w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), self.rope_cache.data_ptr(), pos.data_ptr(),
                          B, T, C, nh, S, st)
            else:
                _hip.call("llj_rmsnorm_rows", w.x.data_ptr(), blk.rms_1.scale.data_ptr(), blk.rms_1.eps,
                          w.xn.data_ptr(), None, M, C, st)
                _hip.call("llj_gemm_qkv_rope", _gz(fa, blk.attn.c_attn), w.xn.data_ptr(), wa.data_ptr(), P(sa), w.q.data_ptr(),
                          kc.data_ptr(), vc.data_ptr(), self.rope_cache.data_ptr(), pos.data_ptr(), B, T, C, nh, S, st)
            self._attention(w, kc, vc, pos, B, T, S, st)
            self._gemm_resid(_gz(fp, blk.attn.c_proj), w.y, wp, sp, w.x, M, C, C, w, st)
            if f1 != f2:
                raise TypeError("c_fc1 and c_fc2 must share a weight format")
            if f1 == 2:
                self._i8_norm_prep(w.x, blk.rms_2, w.xn, M, C, w, st)
                ao, (g1, g2), kp = self._i8_gathered(w.xn, M, C, [(w1, s1, H), (w2, s2, H)], w, st)
                _hip.call("llj_gemm_i8_linear", w.xn.data_ptr(), C, w1.data_ptr(), P(s1), I8ws, P(ao), P(g1), kp,
                          w.h.data_ptr(), H, M, H, C, st)
                _hip.call("llj_gemm_i8_silu_mul", w.xn.data_ptr(), C, w2.data_ptr(), P(s2), I8ws, P(ao), P(g2), kp,
                          w.h.data_ptr(), H, M, H, C, st)
            else:
                _hip.call("llj_rmsnorm_rows", w.x.data_ptr(), blk.rms_2.scale.data_ptr(), blk.rms_2.eps,
                          w.xn.data_ptr(), None, M, C, st)
                g1, g2 = _gz(f1, blk.mlp.c_fc1), _gz(f2, blk.mlp.c_fc2)
                if GEMM_SWIGLU and g1 == g2 == _hip.WF_ZINT and M >= 256 and H % 64 == 0:  # both in one pass
                    # (a partial last wave of tiles: its columns as two K halves, llj_gemm_swiglu_ws)
                    nb = _hip.lib().llj_gemm_swiglu_ws_bytes(g1, M, H, C)
                    if nb:
                        ws = torch.empty(nb // 4, dtype=torch.float32, device=w.h.device)
                        _hip.call("llj_gemm_swiglu_ws", g1, w.xn.data_ptr(), C, w1.data_ptr(), P(s1), w2.data_ptr(),
                                  P(s2), w.h.data_ptr(), H, M, H, C, ws.data_ptr(), nb, st)
                    else:
                        _hip.call("llj_gemm_swiglu", g1, w.xn.data_ptr(), C, w1.data_ptr(), P(s1), w2.data_ptr(),
                                  P(s2), w.h.data_ptr(), H, M, H, C, st)
                else:
                    _hip.call("llj_gemm_linear", g1, w.xn.data_ptr(), C, w1.data_ptr(), P(s1), w.h.data_ptr(), H, M,
                              H, C, st)
                    _hip.call("llj_gemm_silu_mul", g2, w.xn.data_ptr(), C, w2.data_ptr(), P(s2), w.h.data_ptr(), H,
                              M, H, C, st)
            self._gemm_resid(_gz(fd, blk.mlp.c_proj), w.h, wd, sd, w.x, M, C, H, w, st)

    def _gemm_resid(self, f, A, W, sz, x, M, N, K, w, st):
        """x += A . W^T for many rows (LLM.int8: the statistics of A first)."""
        if f == 2:
            self._i8_prep(A, M, K, w, st)
            ao, (wg,), kp = self._i8_gathered(A, M, K, [(W, sz, N)], w, st)
            _hip.call("llj_gemm_i8_resid", A.data_ptr(), A.stride(0), W.data_ptr(), _hip.ptr(sz), _hip.ptr(w.i8ws),
                      _hip.ptr(ao), _hip.ptr(wg), kp, x.data_ptr(), x.stride(0), M, N, K, st)
        else:
            # few row tiles (256..1024 prompt rows): the K range split over workgroups (llj_gemm_resid_ws)
            nb = _hip.lib().llj_gemm_resid_ws_bytes(f, M, N, K) if M >= 256 else 0
            if nb:
                ws = torch.empty(nb // 4, dtype=torch.float32, device=x.device)
                _hip.call("llj_gemm_resid_ws", f, A.data_ptr(), A.stride(0), W.data_ptr(), _hip.ptr(sz), x.data_ptr(),
                          x.stride(0), M, N, K, ws.data_ptr(), nb, st)
            else:
                _hip.call("llj_gemm_resid", f, A.data_ptr(), A.stride(0), W.data_ptr(), _hip.ptr(sz), x.data_ptr(),
                          x.stride(0), M, N, K, st)

    @staticmethod
    def _glinear(spec, A, M, K, N, out, resid, st):
        kind, W, sc, zr, bits, group = spec
        if kind == 2:  # LLM.int8 (Linear8bitLt._gspec): statistics + int8 / fp16 products on f16(A)
            ws = torch.empty(_hip.lib().llj_g_i8_ws_bytes(M, K), dtype=torch.uint8, device=A.device)
            _hip.call("llj_g_i8_linear", A.data_ptr(), A.stride(0), M, K, W.data_ptr(), sc.data_ptr(),
                      Linear8bitLtThreshold, ws.data_ptr(), N, out.data_ptr(), out.stride(0),
                      None if resid is None else resid.data_ptr(), 0 if resid is None else resid.stride(0),
                      _dt_code(A.dtype), st)
            return
        if kind == 1 and W.dtype != A.dtype:
            raise TypeError(f"dense Linear weight {W.dtype} with {A.dtype} activations")
        _hip.call("llj_g_linear", kind, A.data_ptr(), A.stride(0), M, K, W.data_ptr(), _hip.ptr(sc), _hip.ptr(zr), bits,
                  group, N, out.data_ptr(), out.stride(0), None if resid is None else resid.data_ptr(),
                  0 if resid is None else resid.stride(0), _dt_code(A.dtype), st)

    def _blocks_generic(self, w, specs, kv, pos, B, T, S, st):
        """The blocks on the any-shape kernels (csrc/generic.hip), per layer (model.py:162-175):
        rms_1 -> c_attn -> split + RoPE + KV write -> attention -> c_proj + residual -> rms_2 ->
        c_fc1, c_fc2 -> silu * mul -> mlp.c_proj + residual."""
        cfg = self.config
        C, H, nh = cfg.n_embd, MLP.hidden(cfg), cfg.n_head
        M = B * T
        for i, blk in enumerate(self.transformer.h):
            sa, sp, s1, s2, sd = specs["layers"][i]
            kc, vc = kv[i]
            _hip.call("llj_g_rmsnorm", w.x.data_ptr(), C, blk.rms_1.scale.data_ptr(), blk.rms_1.eps, w.xn.data_ptr(), C,
                      M, C, w.dt, st)
            self._glinear(sa, w.xn, M, C, 3 * C, w.qkv, None, st)
            _hip.call("llj_g_rope_kv", w.qkv.data_ptr(), w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                      self.rope_cache.data_ptr(), pos.data_ptr(), B, T, C, nh, S, w.dt, st)
            _hip.call("llj_g_attention", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), w.y.data_ptr(), pos.data_ptr(),
                      B, T, C, nh, S, w.dt, st)
            self._glinear(sp, w.y, M, C, C, w.x, w.x, st)
            _hip.call("llj_g_rmsnorm", w.x.data_ptr(), C, blk.rms_2.scale.data_ptr(), blk.rms_2.eps, w.xn.data_ptr(), C,
                      M, C, w.dt, st)
            self._glinear(s1, w.xn, M, C, H, w.a1, None, st)
            self._glinear(s2, w.xn, M, C, H, w.a2, None, st)
            _hip.call("llj_g_silu_mul", w.a1.data_ptr(), w.a2.data_ptr(), w.h.data_ptr(), M * H, w.dt, st)
            self._glinear(sd, w.h, M, H, C, w.x, w.x, st)

    def _blocks(self, w, specs, kv, pos, B, T, S, st):
        cfg = self.config
        C, H, nh = cfg.n_embd, MLP.hidden(cfg), cfg.n_head
        M = B * T
        rope = self.rope_cache
        P = _hip.ptr
        if w.generic:
            return self._blocks_generic(w, specs, kv, pos, B, T, S, st)
        if w.gemm:
            return self._blocks_gemm(w, specs, kv, pos, B, T, S, st)
        for i, blk in enumerate(self.transformer.h):
            (fa, wa, sa), (fp, wp, sp), (f1, w1, s1), (f2, w2, s2), (fd, wd, sd) = specs["layers"][i]
            kc, vc = kv[i]
            # 1. rms_1 + c_attn + rope + kv write
            rs = None
            if fa == 2 and w.i8s and I8_NORM_ROWSTATS:  # the norm + xn's hand-off block, rows quantized in the GEMV
                _hip.call("llj_i8_norm_rowstats", w.x.data_ptr(), blk.rms_1.scale.data_ptr(), blk.rms_1.eps,
                          w.xn.data_ptr(), M, C, Linear8bitLtThreshold, w.i8ws.data_ptr(), w.n_st.data_ptr(), st)
                _hip.call("llj_norm_qkv_rope", fa | _hip.WF_I8_ROWSTATS, w.xn.data_ptr(), None, blk.rms_1.eps,
                          wa.data_ptr(), P(sa), w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rope.data_ptr(),
                          pos.data_ptr(), B, T, C, nh, S, 0, M, w.n_st.data_ptr(), None, None, 0, st)
                src = None
            elif fa == 2:
                self._i8_norm_prep(w.x, blk.rms_1, w.xn, M, C, w, st)
                src, nw = w.xn, None
            elif w.hand and i > 0:  # the previous mlp.c_proj handed over the sums of squares
                src, nw = w.x, blk.rms_1.scale.data_ptr()
            elif w.pre:
                rs = w.rs if fa in _ROWSUM_FMTS else None
                _hip.call("llj_rmsnorm_rows", w.x.data_ptr(), blk.rms_1.scale.data_ptr(), blk.rms_1.eps,
                          w.xn.data_ptr(), P(rs), M, C, st)
                src, nw = w.xn, None
            else:
                src, nw = w.x, blk.rms_1.scale.data_ptr()
            nst = w.nst if (w.hand and i > 0 and fa != 2) else None
            for r0 in range(0, M if src is not None else 0, QKV_ROWS):
                r = min(QKV_ROWS, M - r0)
                _hip.call("llj_norm_qkv_rope", fa, src.data_ptr(), nw, blk.rms_1.eps, wa.data_ptr(), P(sa),
                          w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rope.data_ptr(), pos.data_ptr(), B, T, C, nh,
                          S, r0, r, P(w.i8ws), P(rs), P(nst), w.npart, st)
            # 2. attention, 3. c_proj + residual
            if w.i8s and not w.flash:  # y's LLM.int8 statistics from the attention (clears h's block)
                _hip.call("llj_attention_i8", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), w.y.data_ptr(), pos.data_ptr(),
                          B, T, nh, C // nh, S, w.nsplit, P(w.att_ws), w.y_st.data_ptr(), w.h_st.data_ptr(),
                          w.h_st.numel(), Linear8bitLtThreshold, st)
                _hip.call("llj_i8_linear_resid", w.y.data_ptr(), C, wp.data_ptr(), P(sp), w.x.data_ptr(), C, M, C, C,
                          w.y_st.data_ptr(), st)
            elif w.att_merge and not w.flash and fp in (0, 1, 3):  # split partials, merged by c_proj (A/B)
                _hip.call("llj_attention_part", w.q.data_ptr(), kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), B, T, nh,
                          C // nh, S, w.att_merge, w.att_part.data_ptr(), st)
                _hip.call("llj_linear_resid_attn", fp, w.att_part.data_ptr(), w.att_merge, nh, wp.data_ptr(), P(sp),
                          w.x.data_ptr(), C, C, C, P(w.nst) if w.hand else None, st)
            else:
                self._attention(w, kc, vc, pos, B, T, S, st)
                self._resid(fp, w.y, wp, sp, w.x, M, C, C, w, st, w.nst if w.hand else None)
            # 4. rms_2 + fc1/fc2 + silu*mul
            if f1 != f2:
                raise TypeError("c_fc1 and c_fc2 must share a weight format")
            rs = None
            if f1 == 2 and w.i8s and I8_NORM_ROWSTATS:
                _hip.call("llj_i8_norm_rowstats", w.x.data_ptr(), blk.rms_2.scale.data_ptr(), blk.rms_2.eps,
                          w.xn.data_ptr(), M, C, Linear8bitLtThreshold, w.i8ws.data_ptr(), w.n_st.data_ptr(), st)
                src, nw, step = w.xn, None, I8_ROWS
            elif f1 == 2:
                self._i8_norm_prep(w.x, blk.rms_2, w.xn, M, C, w, st)
                src, nw, step = w.xn, None, I8_ROWS
            elif w.hand:  # c_proj handed over the sums of squares
                src, nw, step = w.x, blk.rms_2.scale.data_ptr(), QKV_ROWS
            elif w.pre:
                rs = w.rs if f1 in _ROWSUM_FMTS else None
                _hip.call("llj_rmsnorm_rows", w.x.data_ptr(), blk.rms_2.scale.data_ptr(), blk.rms_2.eps,
                          w.xn.data_ptr(), P(rs), M, C, st)
                src, nw, step = w.xn, None, QKV_ROWS
            else:
                src, nw, step = w.x, blk.rms_2.scale.data_ptr(), QKV_ROWS
            nst = w.nst if (w.hand and f1 != 2) else None
            if w.i8s and not w.flash:  # h's LLM.int8 statistics from the SwiGLU (clears y's block)
                ns = I8_NORM_ROWSTATS
                _hip.call("llj_i8_swiglu_stats", src.data_ptr(), w1.data_ptr(), P(s1), w2.data_ptr(), P(s2),
                          w.h.data_ptr(), M, H, C, None if ns else w.i8ws.data_ptr(), w.n_st.data_ptr() if ns else None,
                          w.h_st.data_ptr(), w.y_st.data_ptr(), w.y_st.numel(), Linear8bitLtThreshold, st)
                _hip.call("llj_i8_linear_resid", w.h.data_ptr(), H, wd.data_ptr(), P(sd), w.x.data_ptr(), C, M, C, H,
                          w.h_st.data_ptr(), st)
                continue
            for r0 in range(0, M, step):
                r = min(step, M - r0)
                _hip.call("llj_norm_swiglu", f1, src[r0].data_ptr(), nw, blk.rms_2.eps, w1.data_ptr(), P(s1),
                          w2.data_ptr(), P(s2), w.h[r0].data_ptr(), r, H, C, P(w.i8ws), r0,
                          None if rs is None else rs[r0].data_ptr(), None if nst is None else nst[r0].data_ptr(),
                          w.npart, st)
            # 5. mlp.c_proj + residual
            self._resid(fd, w.h, wd, sd, w.x, M, C, H, w, st, w.nst if w.hand else None)

    def _resid(self, f, A, W, sz, x, M, N, K, w, st, nst=None):
        """x += A . W^T; with `nst` (the norm hand-off, N / 16 tiles x 16 rows) also the next
        RMSNorm's partial sums of squares of the new x."""
        if f == 2:
            self._i8_prep(A, M, K, w, st)
        step = I8_ROWS if f == 2 else LIN_ROWS
        for r0 in range(0, M, step):
            r = min(step, M - r0)
            _hip.call("llj_linear_resid", f, A[r0].data_ptr(), A.stride(0), W.data_ptr(), _hip.ptr(sz),
                      x[r0].data_ptr(), x.stride(0), r, N, K, _hip.ptr(w.i8ws), r0,
                      None if nst is None else nst[r0].data_ptr(), st)

    def _head(self, x, M, specs, out, st, w):
        cfg = self.config
        C, V = cfg.n_embd, cfg.padded_vocab_size
        ln = self.transformer.ln_f
        if w.generic:  # ln_f + lm_head on the any-shape kernels
            xn = w.xn if M <= w.xn.shape[0] else torch.empty_like(x)
            _hip.call("llj_g_rmsnorm", x.data_ptr(), x.stride(0), ln.scale.data_ptr(), ln.eps, xn.data_ptr(), C, M, C,
                      w.dt, st)
            self._glinear(specs["head"], xn, M, C, V, out, None, st)
            return
        f, W, sz = specs["head"]
        rs = nst = None
        if f == 2 and w.i8s and I8_NORM_ROWSTATS and x is w.x:  # ln_f + xn's hand-off block
            xn = w.xn
            _hip.call("llj_i8_norm_rowstats", x.data_ptr(), ln.scale.data_ptr(), ln.eps, xn.data_ptr(), M, C,
                      Linear8bitLtThreshold, w.i8ws.data_ptr(), w.n_st.data_ptr(), st)
            _hip.call("llj_norm_linear", f | _hip.WF_I8_ROWSTATS, xn.data_ptr(), None, ln.eps, W.data_ptr(),
                      _hip.ptr(sz), out.data_ptr(), out.stride(0), M, V, C, w.n_st.data_ptr(), 0, None, None, 0, st)
            return
        if f == 2:
            xn = torch.empty_like(x)
            self._i8_norm_prep(x, ln, xn, M, C, w, st)
            if M >= GEMM_MIN_ROWS and C % 128 == 0 and V % 128 == 0:  # many rows: the int8 GEMM
                ao, (wg,), kp = self._i8_gathered(xn, M, C, [(W, sz, V)], w, st)
                _hip.call("llj_gemm_i8_linear", xn.data_ptr(), C, W.data_ptr(), _hip.ptr(sz), _hip.ptr(w.i8ws),
                          _hip.ptr(ao), _hip.ptr(wg), kp, out.data_ptr(), out.stride(0), M, V, C, st)
                return
            src, nw = xn, None
        elif M >= GEMM_MIN_ROWS and _gemm_fmt(f) and C % 128 == 0 and V % 128 == 0:  # many rows: GEMM
            xn = torch.empty_like(x)
            _hip.call("llj_rmsnorm_rows", x.data_ptr(), ln.scale.data_ptr(), ln.eps, xn.data_ptr(), None, M, C, st)
            _hip.call("llj_gemm_linear", _gz(f, self.lm_head), xn.data_ptr(), C, W.data_ptr(), _hip.ptr(sz),
                      out.data_ptr(), out.stride(0), M, V, C, st)
            return
        elif x is w.x and w.hand and f != 2 and len(self.transformer.h) > 0:  # the last mlp.c_proj's partials
            nst = w.nst
            src, nw = x, ln.scale.data_ptr()
        elif M >= 2 and w.pre:  # batched rows: normalize once (see _Work.pre)
            xn = torch.empty_like(x)
            rs = torch.empty(M, dtype=torch.float32, device=x.device) if f in _ROWSUM_FMTS else None
            _hip.call("llj_rmsnorm_rows", x.data_ptr(), ln.scale.data_ptr(), ln.eps, xn.data_ptr(), _hip.ptr(rs), M,
                      C, st)
            src, nw = xn, None
        else:
            src, nw = x, ln.scale.data_ptr()
        for r0 in range(0, M, QKV_ROWS):
            r = min(QKV_ROWS, M - r0)
            _hip.call("llj_norm_linear", f, src[r0].data_ptr(), nw, ln.eps, W.data_ptr(), _hip.ptr(sz),
                      out[r0].data_ptr(), out.stride(0), r, V, C, _hip.ptr(w.i8ws), r0,
                      None if rs is None else rs[r0].data_ptr(), None if nst is None else nst[r0].data_ptr(),
                      w.npart, st)


Linear8bitLtThreshold = 6.0  # reference quantization.py:45


class Block(nn.Module):
    """reference model.py:154-175 (module tree / parameter names). Its computation runs inside
    LLaMA.forward; a standalone Block.forward is provided for the no-cache case."""

    def __init__(self, config: LLaMAConfig) -> None:
        super().__init__()
        self.rms_1 = RMSNorm(config.n_embd)
        self.attn = CausalSelfAttention(config)
        self.rms_2 = RMSNorm(config.n_embd)
        self.mlp = MLP(config)
        self.config = config

    def forward(self, x, rope, mask, max_seq_length, input_pos=None, kv_cache=None):
        if input_pos is not None or kv_cache is not None:
            raise NotImplementedError("Block.forward with a KV cache runs inside LLaMA.forward(idx, max_seq_length, "
                                      "input_pos) on this path")
        B, T, C = x.shape
        _hip.require_device(x, "x")
        cfg = self.config
        model = _BlockHost(self, cfg)
        return model.run(x, rope), None


class _BlockHost:
    """No-cache Block.forward: the same kernels as LLaMA.forward with positions 0..T-1 and
    `rope` (rows 0..T-1 of the RoPE cache, as the reference passes it) as the table."""

    def __init__(self, blk, cfg):
        self.blk, self.cfg = blk, cfg

    def run(self, x, rope):
        blk, cfg = self.blk, self.cfg
        B, T, C = x.shape
        M = B * T
        mods = (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc1, blk.mlp.c_fc2, blk.mlp.c_proj)
        if cfg.kernel_support() is not None or x.dtype == torch.float32:  # the any-shape kernels
            specs = {"layers": [tuple(_gspec(m) for m in mods)]}
            w = _Work(cfg, M, x.device, False, generic=True, dtype=x.dtype)
        else:
            specs = {"layers": [tuple(_wspec(m) for m in mods)]}
            need_i8 = any(s[0] == 2 for s in specs["layers"][0])
            w = _Work(cfg, M, x.device, need_i8)
        w.x.copy_(x.reshape(M, C))
        kv = [(torch.zeros(B, cfg.n_head, T, C // cfg.n_head, dtype=w.x.dtype, device=x.device),
               torch.zeros(B, cfg.n_head, T, C // cfg.n_head, dtype=w.x.dtype, device=x.device))]
        pos = torch.arange(T, device=x.device, dtype=torch.int32)
        shim = _OneBlock(blk, rope.float().contiguous(), cfg)
        LLaMA._blocks(shim, w, specs, kv, pos, B, T, T, _hip.stream())
        return w.x.view(B, T, C).clone()


class _OneBlock:
    def __init__(self, blk, rope, cfg):
        self.transformer = types.SimpleNamespace(h=[blk])
        self.rope_cache = rope
        self.config = cfg

    def _i8_prep(self, A, M, K, w, st):
        LLaMA._i8_prep(self, A, M, K, w, st)

    def _i8_norm_prep(self, *a):
        LLaMA._i8_norm_prep(self, *a)

    def _resid(self, *a, **kw):
        LLaMA._resid(self, *a, **kw)

    def _gemm_resid(self, *a):
        LLaMA._gemm_resid(self, *a)

    def _attention(self, *a):
        LLaMA._attention(self, *a)

    def _blocks_generic(self, *a):
        LLaMA._blocks_generic(self, *a)

    _glinear = staticmethod(LLaMA._glinear)


class CausalSelfAttention(nn.Module):
    """reference model.py:178-190 (parameters); computed by LLaMA.forward / Block.forward."""

    def __init__(self, config: LLaMAConfig) -> None:
        super().__init__()
        assert config.n_embd % config.n_head == 0
        self.c_attn = nn.Linear(config.n_embd, 3 * config.n_embd, bias=False)
        self.c_proj = nn.Linear(config.n_embd, config.n_embd, bias=False)
        self.n_head = config.n_head
        self.n_embd = config.n_embd
        self.block_size = config.block_size


class MLP(nn.Module):
    """reference model.py:246-260"""

    def __init__(self, config: LLaMAConfig) -> None:
        super().__init__()
        n_hidden = MLP.hidden(config)
        self.c_fc1 = nn.Linear(config.n_embd, n_hidden, bias=False)
        self.c_fc2 = nn.Linear(config.n_embd, n_hidden, bias=False)
        self.c_proj = nn.Linear(n_hidden, config.n_embd, bias=False)

    @staticmethod
    def hidden(config) -> int:
        return find_multiple(int(2 * (4 * config.n_embd) / 3), 256)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _hip.require_device(x, "x")
        K = x.shape[-1]
        x2 = x.reshape(-1, K).contiguous()
        M = x2.shape[0]
        H = self.c_fc1.out_features
        if x.dtype == torch.float32 or K % 128:  # fp32 / any-shape: the generic kernels
            st = _hip.stream()
            a1 = torch.empty(M, H, dtype=x.dtype, device=x.device)
            a2 = torch.empty_like(a1)
            out = torch.empty(M, self.c_proj.out_features, dtype=x.dtype, device=x.device)
            LLaMA._glinear(_gspec(self.c_fc1), x2, M, K, H, a1, None, st)
            LLaMA._glinear(_gspec(self.c_fc2), x2, M, K, H, a2, None, st)
            _hip.call("llj_g_silu_mul", a1.data_ptr(), a2.data_ptr(), a1.data_ptr(), M * H, _dt_code(x.dtype), st)
            LLaMA._glinear(_gspec(self.c_proj), a1, M, H, self.c_proj.out_features, out, None, st)
            return out.view(*x.shape[:-1], out.shape[1])
        (f1, w1, s1), (f2, w2, s2), (fd, wd, sd) = _wspec(self.c_fc1), _wspec(self.c_fc2), _wspec(self.c_proj)
        if f1 != f2:
            raise TypeError("c_fc1 and c_fc2 must share a weight format")
        st = _hip.stream()
        h = torch.empty(M, H, dtype=torch.bfloat16, device=x.device)
        ws = None
        L = _hip.lib()
        if 2 in (f1, fd):
            ws = torch.empty(max(L.llj_i8_ws_bytes(M, K), L.llj_i8_ws_bytes(M, H)), dtype=torch.uint8,
                             device=x.device)
        if f1 == 2:
            _hip.call("llj_i8_stats", x2.data_ptr(), K, M, K, Linear8bitLtThreshold, ws.data_ptr(), st)
        step = I8_ROWS if f1 == 2 else QKV_ROWS
        for r0 in range(0, M, step):
            r = min(step, M - r0)
            _hip.call("llj_norm_swiglu", f1, x2[r0].data_ptr(), None, 0.0, w1.data_ptr(), _hip.ptr(s1), w2.data_ptr(),
                      _hip.ptr(s2), h[r0].data_ptr(), r, H, K, _hip.ptr(ws), r0, None, None, 0, st)
        out = torch.empty(M, self.c_proj.out_features, dtype=torch.bfloat16, device=x.device)
        if fd == 2:
            _hip.call("llj_i8_stats", h.data_ptr(), H, M, H, Linear8bitLtThreshold, ws.data_ptr(), st)
        step = I8_ROWS if fd == 2 else LIN_ROWS
        for r0 in range(0, M, step):
            r = min(step, M - r0)
            _hip.call("llj_linear", fd, h[r0].data_ptr(), H, wd.data_ptr(), _hip.ptr(sd), None, out[r0].data_ptr(),
                      out.stride(0), r, out.shape[1], H, _hip.ptr(ws), r0, None, st)
        return out.view(*x.shape[:-1], out.shape[1])


class RMSNorm(nn.Module):
    """reference model.py:263-283: scale * x * rsqrt(mean(x*x) + eps), bf16 rounding points."""

    def __init__(self, size: int, dim: int = -1, eps: float = 1e-5) -> None:
        super().__init__()
        self.scale = nn.Parameter(torch.ones(size))
        self.eps = eps
        self.dim = dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _hip.require_device(x, "x")
        if x.dtype not in (torch.bfloat16, torch.float32) or self.scale.dtype != x.dtype or self.dim not in (-1, x.dim() - 1):
            raise TypeError("RMSNorm HIP path: bfloat16 (or float32) input and scale over the last dim")
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        y = torch.empty_like(x2)
        if x.dtype == torch.float32:
            _hip.call("llj_g_rmsnorm", x2.data_ptr(), C, self.scale.data_ptr(), self.eps, y.data_ptr(), C, x2.shape[0], C,
                      1, _hip.stream())
            return y.view_as(x)
        _hip.call("llj_rmsnorm", x2.data_ptr(), self.scale.data_ptr(), self.eps, y.data_ptr(), x2.shape[0], C,
                  _hip.stream())
        return y.view_as(x)


def build_rope_cache(seq_len: int, n_elem: int, dtype: torch.dtype, device: torch.device,
                     base: int = 10000) -> RoPECache:
    """reference model.py:286-309 (one-time table; (seq_len, n_elem/2, 2) [cos, sin])."""
    theta = 1.0 / (base ** (torch.arange(0, n_elem, 2, dtype=dtype, device=device) / n_elem))
    seq_idx = torch.arange(seq_len, dtype=dtype, device=device)
    idx_theta = torch.outer(seq_idx, theta).float()
    cache = torch.stack([torch.cos(idx_theta), torch.sin(idx_theta)], dim=-1)
    if dtype in (torch.float16, torch.bfloat16, torch.int8):
        cache = cache.half()
    return cache


def apply_rope(x: torch.Tensor, rope_cache: RoPECache) -> torch.Tensor:
    """reference model.py:312-329. On this path RoPE is fused into the c_attn epilogue
    (llj_norm_qkv_rope); this standalone form is the reference's definition."""
    T = x.size(1)
    rope_cache = rope_cache[:T]
    xshaped = x.float().reshape(*x.shape[:-1], -1, 2)
    rope_cache = rope_cache.view(1, xshaped.size(1), 1, xshaped.size(3), 2)
    x_out2 = torch.stack(
        [
            xshaped[..., 0] * rope_cache[..., 0] - xshaped[..., 1] * rope_cache[..., 1],
            xshaped[..., 1] * rope_cache[..., 0] + xshaped[..., 0] * rope_cache[..., 1],
        ],
        -1,
    )
    return x_out2.flatten(3).type_as(x)
