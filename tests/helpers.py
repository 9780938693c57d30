"""Shared test helpers: host-side statements of the device layouts and tolerance rules."""
import numpy as np

from oracle import llama_np as O


def w4p_pack_np(qw_logical: np.ndarray) -> np.ndarray:
    """Host restatement of the W4P layout (csrc/w4pack.hip) from the reference's logical
    (N, K/2) int4 byte array. Returns the packed bytes as uint8 (N*K/2,)."""
    N, Kh = qw_logical.shape
    K = 2 * Kh
    q = O.colblock_unpack_q(qw_logical, 4).astype(np.uint32)  # (N, K) codes
    KC = K // 128
    # index tiles: [nt][kc][lane][t] dwords; lane = 16*g + n_local; codes k = 128kc + 32g + 8t + j
    q = q.reshape(N // 16, 16, KC, 4, 4, 8)  # nt, n_local, kc, g, t, j
    bits = np.array([4 * (j >> 1) + 16 * (j & 1) for j in range(8)], np.uint32)
    d = (q << bits).sum(-1, dtype=np.uint64).astype(np.uint32)  # nt, n_local, kc, g, t
    d = d.transpose(0, 2, 3, 1, 4)  # nt, kc, g, n_local, t
    return np.ascontiguousarray(d).reshape(-1).view(np.uint8)


def w8p_pack_np(qw_logical: np.ndarray) -> np.ndarray:
    """Host restatement of the W8P layout (csrc/w4pack.hip) from the reference's logical (N, K)
    int8-code byte array (ColBlock bits=8): per (16-column tile, 128-k chunk) the W4P tile of
    the low nibbles, then the W4P tile of the high nibbles. Returns uint8 (N*K,)."""
    N, K = qw_logical.shape

    def as_w4_logical(nib):  # (N, K) nibbles -> the (N, K/2) int4 byte array of the same codes
        return (nib[:, 0::2] | (nib[:, 1::2] << 4)).astype(np.uint8)

    lo = w4p_pack_np(as_w4_logical(qw_logical & 0xF)).reshape(-1, 1024)
    hi = w4p_pack_np(as_w4_logical(qw_logical >> 4)).reshape(-1, 1024)
    return np.ascontiguousarray(np.stack([lo, hi], 1)).reshape(-1)


def bf16(x):
    return O.bf16_round(np.asarray(x, np.float32))


def assert_bf16_close(got, ref, what="", rel=1.2e-2, abs_frac=4e-3):
    """bf16 outputs against an fp32 reference: per element |d| <= rel*|ref| + abs_frac*max|ref|
    (one bf16 rounding of the output is 2^-9 relative; accumulation-order noise is far below)."""
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    scale = float(np.abs(ref).max()) or 1.0
    err = np.abs(got - ref)
    bound = rel * np.abs(ref) + abs_frac * scale
    bad = err > bound
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} outside bf16 tolerance; max err {err.max():.4g} (scale {scale:.4g})"
