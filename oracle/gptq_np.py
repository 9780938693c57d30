"""numpy restatement of the reference GPTQ producer — TEST INFRASTRUCTURE (see oracle/__init__.py).

Follows /root/reference/lit_llama/quantization.py:424-614 (GPTQQuantizer, the IST-DASLab GPTQ
algorithm, arXiv:2210.17323) for the configuration quantize/gptq.py:84-90 uses for gptq.int4 /
gptq.int8: per-channel, asymmetric, blocksize 128, percdamp 0.01, groupsize -1, actorder True;
and grouped scales (groupsize g, actorder off; 571-577). The reference's own grouped column loop
raises (576 assigns the (N, 1) scale into the (N,) column scales[:, j]), so the grouped case
restates the algorithm as written there (a group's (scale, zero) from find_params_weight on the
group's columns of W as updated by the earlier blocks, at the group's first column) and its
parity is UNPINNED: no reference output exists (tests/golden/make_golden.py gen_gptq_grouped).
Every step is fp32 like the reference's torch CPU run; the column loop is the reference's op
order with each fp32 op rounded on its own (numpy does not contract to FMA), so it is bitwise
the reference's loop given the same W1 / Hinv1. The Cholesky factors come from LAPACK in fp32 as
torch's do, but not necessarily the same LAPACK build: the end-to-end comparison against the
reference's own output (tests/golden/gptq.npz) allows rare code flips (see tests/test_gptq.py).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

F32 = np.float32


def find_params_weight(W: np.ndarray, bits: int, perchannel: bool = True, sym: bool = False):
    """quantization.py:475-514: per-row (scale, zero) (perchannel), or one pair for the whole matrix
    repeated per row (perchannel=False, 481-482 / 503-506); sym: the range symmetric about 0
    (488-492) and zero = (maxq + 1) / 2 (498-499)."""
    maxq = F32(2 ** bits - 1)
    x = W.astype(F32)
    if not perchannel:
        x = x.reshape(1, -1)
    xmin = np.minimum(x.min(1), F32(0))
    xmax = np.maximum(x.max(1), F32(0))
    if sym:
        xmax = np.maximum(np.abs(xmin), xmax).astype(F32)
        xmin = np.where(xmin < 0, -xmax, xmin).astype(F32)
    both0 = (xmin == 0) & (xmax == 0)
    xmin = np.where(both0, F32(-1), xmin).astype(F32)
    xmax = np.where(both0, F32(1), xmax).astype(F32)
    scale = ((xmax - xmin) / maxq).astype(F32)
    if sym:
        zero = np.full_like(scale, (maxq + 1) / 2).astype(F32)
    else:
        zero = np.round(-xmin / scale).astype(F32)  # np.round is half-to-even like torch.round
    if not perchannel:
        scale, zero = np.repeat(scale, W.shape[0]), np.repeat(zero, W.shape[0])
    return scale, zero


def collect_input_stats(H: np.ndarray, nsamples: int, inp: np.ndarray):
    """quantization.py:516-530: running H = 2/n Σ x xᵀ over the calibration samples of one call
    (inp (B, T, K) or (T, K)). Returns (H, nsamples)."""
    if inp.ndim == 2:
        inp = inp[None]
    tmp = inp.shape[0]
    x = inp.reshape(-1, inp.shape[-1]).T.astype(F32)
    H = (H * F32(nsamples / (nsamples + tmp))).astype(F32)
    nsamples += tmp
    x = (F32(np.sqrt(2 / nsamples)) * x).astype(F32)
    return (H + x @ x.T).astype(F32), nsamples


def hinv_upper(H: np.ndarray, actorder: bool = True, percdamp: float = 0.01):
    """quantization.py:540-564: dead columns, act-order permutation, dampening, then
    cholesky -> cholesky_inverse -> upper cholesky. Returns (Hinv (K, K) fp32, perm or None, dead)."""
    H = H.astype(F32).copy()
    K = H.shape[0]
    dead = np.diag(H) == 0
    H[dead, dead] = 1
    perm = None
    if actorder:
        perm = np.argsort(-np.diag(H), kind="stable")
        H = H[perm][:, perm]
    damp = F32(percdamp) * F32(np.mean(np.diag(H), dtype=F32))
    H[np.arange(K), np.arange(K)] += damp
    L = np.linalg.cholesky(H).astype(F32)
    Li = scipy.linalg.solve_triangular(L, np.eye(K, dtype=F32), lower=True).astype(F32)
    Hi = (Li.T @ Li).astype(F32)  # cholesky_inverse(L) = (L Lᵀ)⁻¹
    U = np.ascontiguousarray(np.linalg.cholesky(Hi).T, dtype=F32)  # upper factor: Hi = Uᵀ U
    return U, perm, dead


def gptq_block(W1: np.ndarray, Hinv1: np.ndarray, scale, zero, bits: int):
    """quantization.py:568-596 for one block, in place on a copy of W1 (N, count). scale / zero:
    (N,) for the whole block, or (N, count) per column (grouped). Returns (Q1 reconstructions,
    Err1, Losses1) — each op fp32, the reference's order."""
    maxq = F32(2 ** bits - 1)
    W1 = W1.astype(F32).copy()
    N, count = W1.shape
    Q1 = np.zeros_like(W1)
    Err1 = np.zeros_like(W1)
    L1 = np.zeros_like(W1)
    for i in range(count):
        w = W1[:, i].copy()
        d = Hinv1[i, i]
        sc = scale if np.ndim(scale) == 1 else scale[:, i]
        zr = zero if np.ndim(zero) == 1 else zero[:, i]
        q = np.clip(np.round(w / sc).astype(F32) + zr, F32(0), maxq).astype(F32)  # 470-473
        q = (sc * (q - zr)).astype(F32)
        Q1[:, i] = q
        dq = (w - q).astype(F32)
        L1[:, i] = (dq * dq).astype(F32) / F32(d * d)
        e = (dq / d).astype(F32)
        W1[:, i:] = (W1[:, i:] - (e[:, None] * Hinv1[i, i:][None, :]).astype(F32)).astype(F32)
        Err1[:, i] = e
    return Q1, Err1, L1


def gptq_quantize(W: np.ndarray, H: np.ndarray, bits: int, blocksize: int = 128, actorder: bool = True,
                  percdamp: float = 0.01, groupsize: int = -1, perchannel: bool = True, sym: bool = False):
    """GPTQQuantizer.quantize (quantization.py:532-614). W (N, K) fp32, H (K, K). Returns
    (Q reconstructions (N, K), scale, zero, error) with scale / zero (N,) for groupsize -1, else
    (N, ceil(K / groupsize)) (see the module header: grouped parity unpinned)."""
    assert not (actorder and groupsize != -1)  # 465-467
    W = W.astype(F32).copy()
    scale, zero = find_params_weight(W, bits, perchannel, sym)
    K0 = W.shape[1]
    if groupsize != -1:
        G = (K0 + groupsize - 1) // groupsize
        scales = np.repeat(scale[:, None], G, 1)  # self.scales[:] = scale (533)
        zeros = np.repeat(zero[:, None], G, 1)
    Hinv, perm, dead = hinv_upper(H, actorder, percdamp)
    W[:, dead] = 0
    if perm is not None:
        W = W[:, perm]
    N, K = W.shape
    Q = np.zeros_like(W)
    Losses = np.zeros_like(W)
    cur = (scale, zero)
    for i1 in range(0, K, blocksize):
        i2 = min(i1 + blocksize, K)
        bs, bz = scale, zero
        if groupsize != -1:  # 571-577: params at each group's first column, from W before this block's loop
            bs, bz = np.empty((N, i2 - i1), F32), np.empty((N, i2 - i1), F32)
            for i in range(i2 - i1):
                c = i1 + i
                if c % groupsize == 0:
                    cur = find_params_weight(W[:, c:c + groupsize], bits, perchannel, sym)
                    scales[:, c // groupsize], zeros[:, c // groupsize] = cur
                bs[:, i], bz[:, i] = cur
        Q1, Err1, L1 = gptq_block(W[:, i1:i2], Hinv[i1:i2, i1:i2], bs, bz, bits)
        Q[:, i1:i2] = Q1
        Losses[:, i1:i2] = L1 / F32(2)
        W[:, i2:] = (W[:, i2:] - (Err1 @ Hinv[i1:i2, i2:]).astype(F32)).astype(F32)
    if perm is not None:
        Q = Q[:, np.argsort(perm)]
    if groupsize != -1:
        return Q, scales, zeros, float(Losses.sum())
    return Q, scale, zero, float(Losses.sum())


def pack_weight(Q: np.ndarray, scale, zero, bits: int, tile_cols: int = -1) -> np.ndarray:
    """ColBlockQuantizedLinear.pack_weight (quantization.py:374-388): codes =
    uint8(clamp(Q / scale + zero, 0, 2^bits - 1)) (truncating), packed entries_per_byte per byte,
    column epb*j + nr at bit nr*bits; scale / zero (N,) or (N, groups) with tile_cols columns per
    group. Returns quant_weight as its logical (N, K/epb) array."""
    epb = 8 // bits
    K = Q.shape[1]
    if np.ndim(scale) == 1:
        scale, zero, tile_cols = scale[:, None], zero[:, None], K
    tc = K if tile_cols == -1 else tile_cols
    col = np.arange(K) // tc
    c = np.clip((Q / scale[:, col]).astype(F32) + zero[:, col], 0, 2 ** bits - 1).astype(F32)
    codes = c.astype(np.uint8)
    out = np.zeros((Q.shape[0], Q.shape[1] // epb), np.uint8)
    for nr in range(epb):
        out += (codes[:, nr::epb] << (nr * bits)).astype(np.uint8)
    return out
