"""numpy restatement of the reference LLaMA decode path — TEST INFRASTRUCTURE (see oracle/__init__.py).

All citations are to /root/reference (if001/lit-llama-ja). Everything computes in fp32
(what the reference runs on a CPU host, generate.py:121) unless a function says otherwise.
"""
from __future__ import annotations

import math

import numpy as np

from .weights import Cfg

F32 = np.float32


# ------------------------------------------------------------------ numerics helpers
def bf16_round(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 -> fp32, round-to-nearest-even (torch's .to(torch.bfloat16))."""
    x = np.ascontiguousarray(x, dtype=F32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(F32)
    return np.where(np.isnan(x), x, out)


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    return (bf16_round(x).view(np.uint32) >> 16).astype(np.uint16)


def from_bf16_bits(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(F32)


# ------------------------------------------------------------------ elementwise ops
def build_rope_cache(seq_len: int, n_elem: int, base: int = 10000) -> np.ndarray:
    """reference lit_llama/model.py:286-309, as called with dtype=idx.dtype (int) from
    LLaMA.build_rope_cache (134-140): theta/arange divide in fp32, cache fp32 (seq, n/2, 2)."""
    ar = np.arange(0, n_elem, 2, dtype=np.int64).astype(F32) / F32(n_elem)
    theta = (F32(1.0) / (F32(base) ** ar)).astype(F32)
    seq_idx = np.arange(seq_len, dtype=np.int64).astype(F32)
    idx_theta = np.outer(seq_idx, theta).astype(F32)
    return np.stack([np.cos(idx_theta), np.sin(idx_theta)], axis=-1).astype(F32)


def apply_rope(x: np.ndarray, rope: np.ndarray) -> np.ndarray:
    """reference model.py:312-329. x (B, T, nh, hs); rope (T, hs/2, 2); interleaved pairs."""
    B, T, nh, hs = x.shape
    xs = x.astype(F32).reshape(B, T, nh, hs // 2, 2)
    r = rope[:T].reshape(1, T, 1, hs // 2, 2)
    o0 = xs[..., 0] * r[..., 0] - xs[..., 1] * r[..., 1]
    o1 = xs[..., 1] * r[..., 0] + xs[..., 0] * r[..., 1]
    return np.stack([o0, o1], -1).reshape(B, T, nh, hs).astype(F32)


def rmsnorm(x: np.ndarray, scale: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    """reference model.py:276-283: scale * x * rsqrt(mean(x*x) + eps)."""
    x = x.astype(F32)
    ms = np.mean(x * x, axis=-1, keepdims=True, dtype=F32)
    return (scale.astype(F32) * (x * (F32(1.0) / np.sqrt(ms + F32(eps))))).astype(F32)


def rmsnorm_bf16(x: np.ndarray, scale: np.ndarray, eps: float = 1e-5, cpu_rsqrt: bool = False) -> np.ndarray:
    """reference model.py:276-283 evaluated on bf16 tensors (the reference's GPU precision): every
    torch op rounds its result to bf16 -- x*x, mean (fp32 accumulation inside), + eps, rsqrt,
    x * r, scale * x_normed. rsqrt is one rounding of the fp32 value (the CUDA kernel); torch's
    CPU bf16 rsqrt instead rounds sqrt first and then the reciprocal (cpu_rsqrt=True, which
    reproduces the reference's bf16 CPU output bit for bit, tests/test_oracle_golden.py)."""
    x = bf16_round(x)
    xx = bf16_round(x * x)
    ms = bf16_round(np.mean(xx, axis=-1, keepdims=True, dtype=F32))
    e = bf16_round(ms + F32(eps))
    r = bf16_round(F32(1.0) / (bf16_round(np.sqrt(e)) if cpu_rsqrt else np.sqrt(e)))
    return bf16_round(bf16_round(scale.astype(F32)) * bf16_round(x * r))


def silu(x: np.ndarray) -> np.ndarray:
    x = x.astype(F32)
    return (x / (F32(1.0) + np.exp(-x))).astype(F32)


# ------------------------------------------------------------------ ColBlockQuantizedLinear
def colblock_pack(weight: np.ndarray, scales: np.ndarray, zeros: np.ndarray, bits: int,
                  tile_cols: int = -1) -> np.ndarray:
    """reference quantization.py:374-388 (pack_weight). Returns the LOGICAL (N, K/epb) uint8
    array: byte[:, j] = sum_nr w[:, epb*j+nr] << (nr*bits) (even column -> low nibble)."""
    N, K = weight.shape
    tc = K if tile_cols == -1 else tile_cols
    epb = 8 // bits
    w = weight.astype(F32).copy()
    for j in range(scales.shape[1]):
        w[:, j * tc:(j + 1) * tc] /= scales[:, j:j + 1]
        w[:, j * tc:(j + 1) * tc] += zeros[:, j:j + 1]
    # torch .to(uint8) truncates toward zero after the clamp
    wq = np.clip(w, 0, 2 ** bits - 1).astype(np.uint8)
    out = np.zeros((N, K // epb), np.uint8)
    for nr in range(epb):
        out += (wq[:, nr::epb] << (nr * bits)).astype(np.uint8)
    return out


def colblock_unpack_q(qw: np.ndarray, bits: int) -> np.ndarray:
    """Integer codes q[n, k] from the logical (N, K/epb) byte array (get_weight 396-400)."""
    N, Kb = qw.shape
    epb = 8 // bits
    mask = (1 << bits) - 1
    q = np.empty((N, Kb * epb), np.uint8)
    for nr in range(epb):
        q[:, nr::epb] = (qw >> (nr * bits)) & mask
    return q


def colblock_get_weight(qw, scales, zeros, bits: int, tile_cols: int = -1, bf16: bool = False):
    """reference quantization.py:390-409: (q - zero) * scale per tile, in fp32 (or with the
    bf16 rounding the bf16 CPU fallback applies after each op when bf16=True)."""
    q = colblock_unpack_q(qw, bits).astype(F32)
    N, K = q.shape
    tc = K if tile_cols == -1 else tile_cols
    for j in range(scales.shape[1]):
        sl = slice(j * tc, (j + 1) * tc)
        q[:, sl] -= zeros[:, j:j + 1].astype(F32)
        if bf16:
            q[:, sl] = bf16_round(q[:, sl])
        q[:, sl] *= scales[:, j:j + 1].astype(F32)
        if bf16:
            q[:, sl] = bf16_round(q[:, sl])
    return q


def qlinear_4bit(x: np.ndarray, qw: np.ndarray, scales: np.ndarray, zeros: np.ndarray) -> np.ndarray:
    """Triton GPU path, reference quantization.py:282-331 and 250-267: fp32 A, fp32
    b = ((byte >> 4*(k%2)) & 0xF - zero) * scale, fp32 dot. One (scale, zero) per row."""
    W = colblock_get_weight(qw, scales, zeros, 4)
    return (x.astype(F32).reshape(-1, x.shape[-1]) @ W.T).reshape(*x.shape[:-1], W.shape[0])


# ------------------------------------------------------------------ LLM.int8() (unpinned)
def int8_quantize_weight(w: np.ndarray):
    """bnb.functional.double_quant(W.half()) as used by reference quantization.py:67-75:
    row-wise absmax. CB[n,k] = round(W16[n,k] * 127 / SCB[n]) int8, SCB fp32 (N,).
    Restated from the published LLM.int8() algorithm (bitsandbytes absent: parity unpinned)."""
    w16 = w.astype(np.float16).astype(F32)
    scb = np.abs(w16).max(axis=1).astype(F32)
    safe = np.where(scb == 0, F32(1.0), scb)
    cb = np.rint(w16 * (F32(127.0) / safe[:, None])).clip(-127, 127).astype(np.int8)
    return cb, scb


def int8_linear(x: np.ndarray, cb: np.ndarray, scb: np.ndarray, threshold: float = 6.0) -> np.ndarray:
    """LLM.int8() matmul (bnb MatMul8bitLt, has_fp16_weights=False, threshold=6.0 as set by
    reference quantization.py:45), restated:
      A16 = A.half(); outlier columns = {k : any row |A16[m,k]| >= threshold}
      SCA[m] = absmax over the row's non-outlier elements; CA = round(A16*127/SCA), with
      outlier columns zeroed; out = f16(f16((CA @ CB^T)_int32 * SCA*SCB/127^2)
      + A16[:, outl] @ f16(CB[:, outl]*SCB/127)^T)   (mm_dequant writes fp16; the fp16 side product
      is fp32-accumulated and added to it in one fp16 rounding -- the rounding points of the decode /
      prefill kernels, csrc/gemv_impl.h mm_dequant epilogue; bitsandbytes is unpinned, so which fp16
      points its own MatMul8bitLt used cannot be checked here).
    Returns fp32 holding fp16 values (the caller casts back to the activation dtype)."""
    A = x.astype(F32).reshape(-1, x.shape[-1])
    a16 = A.astype(np.float16).astype(F32)
    big = np.abs(a16) >= threshold
    outl = np.nonzero(big.any(axis=0))[0]
    inl = np.where(big, F32(0.0), a16)
    sca = np.abs(inl).max(axis=1).astype(F32)
    safe = np.where(sca == 0, F32(1.0), sca)
    ca = np.rint(inl * (F32(127.0) / safe[:, None])).clip(-127, 127)
    ca[:, outl] = 0
    # int32-range accumulation, exact in float64 (|sum| <= 127^2 * K < 2^53) and BLAS-fast
    acc = ca.astype(np.float64) @ cb.astype(np.float64).T
    out = (acc.astype(F32) * (sca[:, None] * scb[None, :] / F32(127.0 * 127.0))).astype(np.float16).astype(F32)
    if outl.size:
        wsub = (cb[:, outl].astype(F32) * (scb[:, None] / F32(127.0))).astype(np.float16).astype(F32)
        out = (out + a16[:, outl] @ wsub.T).astype(F32)
    out = out.astype(np.float16).astype(F32)
    return out.reshape(*x.shape[:-1], cb.shape[0]).astype(F32)


# ------------------------------------------------------------------ model
class LinearSpec:
    """What a Linear holds: dense fp32 weight, ColBlock int4/int8 packed, or LLM.int8."""

    def __init__(self, kind: str, **kw):
        self.kind = kind
        self.__dict__.update(kw)

    def __call__(self, x: np.ndarray) -> np.ndarray:
        if self.kind == "dense":
            return (x.astype(F32) @ self.w.T).astype(F32)
        if self.kind == "colblock":
            if not hasattr(self, "_wdeq"):
                self._wdeq = colblock_get_weight(self.qw, self.scales, self.zeros, self.bits,
                                                 getattr(self, "tile_cols", -1))
            return (x.astype(F32) @ self._wdeq.T).astype(F32)
        if self.kind == "int8":
            return int8_linear(x, self.cb, self.scb)
        raise ValueError(self.kind)


class OracleLLaMA:
    """reference lit_llama/model.py:59-151 with the KV-cache path (input_pos given)."""

    def __init__(self, cfg: Cfg, params: dict, linears: dict | None = None, act_bf16: bool = False,
                 cpu_rsqrt: bool = False):
        self.cfg = cfg
        self.p = params
        self.act_bf16 = act_bf16  # round activations to bf16 at module boundaries
        self.cpu_rsqrt = cpu_rsqrt  # bf16 RMSNorm with torch's CPU rsqrt (see rmsnorm_bf16)
        self.lin = {}
        for name in [k[:-len(".weight")] for k in params if k.endswith(".weight") and "wte" not in k]:
            self.lin[name] = LinearSpec("dense", w=params[name + ".weight"].astype(F32))
        if linears:
            self.lin.update(linears)
        self.rope = build_rope_cache(cfg.block_size, cfg.head_size)
        self.kv = None

    def _r(self, x):
        return bf16_round(x) if self.act_bf16 else x

    def _norm(self, x, scale):
        return rmsnorm_bf16(x, scale, cpu_rsqrt=self.cpu_rsqrt) if self.act_bf16 else rmsnorm(x, scale)

    def reset_cache(self):
        """reference model.py:146-151"""
        self.kv = None

    def forward(self, idx: np.ndarray, max_seq_length: int | None = None, input_pos=None) -> np.ndarray:
        """reference model.py:84-128"""
        cfg = self.cfg
        B, T = idx.shape
        S = cfg.block_size if max_seq_length is None else max_seq_length
        assert T <= S <= cfg.block_size
        if input_pos is not None:
            input_pos = np.asarray(input_pos, dtype=np.int64)
            rope = self.rope[input_pos]
            tril = np.tril(np.ones((cfg.block_size, cfg.block_size), bool))
            mask = tril[input_pos][:, :S]
        else:
            rope = self.rope[:T]
            mask = np.tril(np.ones((T, T), bool))
        x = self._r(self.p["transformer.wte.weight"][idx].astype(F32))
        if input_pos is not None and self.kv is None:
            hs = cfg.head_size
            self.kv = [[np.zeros((B, cfg.n_head, S, hs), F32), np.zeros((B, cfg.n_head, S, hs), F32)]
                       for _ in range(cfg.n_layer)]
        for i in range(cfg.n_layer):
            x = self._block(i, x, rope, mask, S, input_pos)
        x = self._norm(x, self.p["transformer.ln_f.scale"])
        return self._r(self.lin["lm_head"](x))

    __call__ = forward

    def _block(self, i, x, rope, mask, S, input_pos):
        """reference model.py:162-175 + CausalSelfAttention 192-243 + MLP 257-260"""
        cfg, p, pre = self.cfg, self.p, f"transformer.h.{i}."
        B, T, C = x.shape
        nh, hs = cfg.n_head, cfg.head_size
        h = self._norm(x, p[pre + "rms_1.scale"])
        qkv = self._r(self.lin[pre + "attn.c_attn"](h))
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        q = self._r(apply_rope(q.reshape(B, T, nh, hs), rope)).transpose(0, 2, 1, 3)
        k = self._r(apply_rope(k.reshape(B, T, nh, hs), rope)).transpose(0, 2, 1, 3)
        v = v.reshape(B, T, nh, hs).transpose(0, 2, 1, 3)
        if input_pos is not None:
            ck, cv = self.kv[i]
            pos = input_pos
            if pos[-1] >= S:  # model.py:221-225: roll left once, write at S-1
                pos = np.array([S - 1])
                ck = np.roll(ck, -1, axis=2)
                cv = np.roll(cv, -1, axis=2)
            ck = ck.copy(); cv = cv.copy()
            ck[:, :, pos] = k
            cv[:, :, pos] = v
            self.kv[i] = [ck, cv]
            k, v = ck, cv
        att = (q @ k.transpose(0, 1, 3, 2)) * F32(1.0 / math.sqrt(hs))
        att = np.where(mask[None, None], att, -np.inf)
        att = att - att.max(-1, keepdims=True)
        e = np.exp(att)
        a = e / e.sum(-1, keepdims=True)
        y = (a @ v).astype(F32).transpose(0, 2, 1, 3).reshape(B, T, C)
        y = self._r(y)
        x = self._r(x + self._r(self.lin[pre + "attn.c_proj"](y)))
        h = self._norm(x, p[pre + "rms_2.scale"])
        a1 = self._r(self.lin[pre + "mlp.c_fc1"](h))
        a2 = self._r(self.lin[pre + "mlp.c_fc2"](h))
        m = self._r(self._r(silu(a1)) * a2)
        return self._r(x + self._r(self.lin[pre + "mlp.c_proj"](m)))


def generate_greedy(model: OracleLLaMA, idx: np.ndarray, max_new_tokens: int, *,
                    max_seq_length: int | None = None, eos_id: int | None = None,
                    return_logits: bool = False):
    """reference generate.py:18-89 with top_k=1 (greedy; multinomial over a one-hot is
    deterministic). idx is 1-D (batch 1, generate.py:62). EOS returns idx[:input_pos], which
    EXCLUDES the EOS token (generate.py:86-87)."""
    T = idx.shape[0]
    T_new = T + max_new_tokens
    if max_seq_length is None:
        max_seq_length = min(T_new, model.cfg.block_size)
    out = np.empty(T_new, np.int32)
    out[:T] = idx
    input_pos = np.arange(T)
    logits_trace = []
    for _ in range(max_new_tokens):
        x = out[input_pos][None]
        logits = model.forward(x, max_seq_length, input_pos)[0, -1]
        logits_trace.append(logits)
        nxt = int(np.argmax(logits))
        input_pos = input_pos[-1:] + 1
        out[input_pos[0]] = nxt
        if eos_id is not None and nxt == eos_id:
            out = out[:input_pos[0]]
            break
    model.reset_cache()
    return (out, np.stack(logits_trace)) if return_logits else out


def topk_filter(logits: np.ndarray, top_k: int, temperature: float = 1.0) -> np.ndarray:
    """reference generate.py:66-73: logits/temperature, keep >= k-th largest, softmax."""
    l = logits.astype(F32) / F32(temperature)
    v = np.sort(l)[::-1][min(top_k, l.shape[-1]) - 1]
    l = np.where(l < v, -np.inf, l)
    e = np.exp(l - l.max())
    return e / e.sum()


def sample_inverse_cdf(logits: np.ndarray, temperature: float, top_k: int | None, u: float):
    """reference generate.py:66-74 on a bf16 logits row (its GPU precision), with the draw of
    torch.multinomial written as an inverse CDF at the uniform u (any exact sampler of the same
    probabilities is the reference's distribution; torch's own generator stream cannot be
    reproduced): x = bf16(logits * (1 / temperature)); keep x >= the top_k-th largest x (ties
    kept); probs = bf16(exp(x - max) * (1 / sum)); return (first index whose running sum of probs
    in index order exceeds u * sum(probs), probs)."""
    x = bf16_round(bf16_round(logits).astype(F32) * F32(1.0 / temperature))
    V = x.shape[-1]
    k = V if top_k is None or top_k < 1 or top_k > V else top_k
    thr = np.sort(x)[::-1][k - 1]
    keep = x >= thr
    xmax = x.max()
    e = np.where(keep, np.exp((x - xmax).astype(F32)), F32(0)).astype(F32)
    tot = F32(e.sum(dtype=F32))
    p = np.where(keep, bf16_round(e * (F32(1.0) / tot)), F32(0)).astype(F32)
    cdf = np.cumsum(p, dtype=F32)
    target = F32(u) * cdf[-1]
    hit = np.nonzero(cdf > target)[0]
    idx = int(hit[0]) if hit.size else int(np.nonzero(keep)[0][-1])
    return idx, p


def sample_inverse_cdf_fp32(logits: np.ndarray, temperature: float, top_k: int | None, u: float):
    """reference generate.py:66-74 on a float32 logits row (its float32 model, generate.py:121 on a
    host without bf16): x = logits / temperature in fp32; keep x >= the top_k-th largest (ties kept);
    probs = exp(x - max) * (1 / sum) in fp32 (torch's softmax up to its exp / summation rounding);
    the inverse-CDF draw at u as sample_inverse_cdf. Returns (index, probs)."""
    x = (logits.astype(F32) / F32(temperature)).astype(F32)
    V = x.shape[-1]
    k = V if top_k is None or top_k < 1 or top_k > V else top_k
    thr = np.sort(x)[::-1][k - 1]
    keep = x >= thr
    e = np.where(keep, np.exp((x - x.max()).astype(F32)), F32(0)).astype(F32)
    p = np.where(keep, e * (F32(1.0) / F32(e.sum(dtype=F32))), F32(0)).astype(F32)
    cdf = np.cumsum(p, dtype=F32)
    hit = np.nonzero(cdf > F32(u) * cdf[-1])[0]
    idx = int(hit[0]) if hit.size else int(np.nonzero(keep)[0][-1])
    return idx, p
