"""Kernel-level parity of the HIP library against the numpy oracle (GPU only).

Every call goes through the C ABI (_lljamd.so via ctypes). Inputs are seeded; expected
values come from oracle/llama_np.py (CPU restatement of the reference, pinned by
tests/test_oracle_golden.py) or from the reference's own fixtures in tests/golden/.
Tolerances: int/byte work is bit-exact; bf16 outputs within one bf16 rounding (see
helpers.assert_bf16_close).
"""
import numpy as np
import pytest
import torch

from lit_llama import _hip
from oracle import llama_np as O
from tests.helpers import assert_bf16_close, bf16, w4p_pack_np, w8p_pack_np

pytestmark = pytest.mark.gpu
dev = "cuda"


def T(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def st():
    return torch.cuda.current_stream().cuda_stream


class option:
    """llj_set_option for the duration of a `with` block (host-side A/B options)."""

    def __init__(self, hip, which, value):
        self.hip, self.which, self.value = hip, which, value

    def __enter__(self):
        self.old = self.hip.llj_set_option(self.which, self.value)
        assert self.old != -1000

    def __exit__(self, *exc):
        self.hip.llj_set_option(self.which, self.old)


def call(hip, name, *args):
    rc = getattr(hip, name)(*args)
    assert rc == 0, f"{name} returned {rc}"


def rand_w4(rng, N, K):
    qw = rng.integers(0, 256, size=(N, K // 2), dtype=np.uint8)
    scales = rng.uniform(0.5, 1.5, size=(N, 1)).astype(np.float32) * np.float32(0.02 / 7)
    zeros = rng.integers(0, 16, size=(N, 1)).astype(np.float32)
    return qw, scales, zeros


def repack(hip, qw):
    N, Kh = qw.shape
    ref = T(qw.T.copy())  # physical (K/2, N) row-major = the reference's column-major buffer
    out = torch.empty(N * Kh, dtype=torch.uint8, device=dev)
    call(hip, "llj_w4_repack", ref.data_ptr(), out.data_ptr(), N, 2 * Kh, st())
    return out


def sz_of(hip, scales, zeros, bits=4):
    N = scales.shape[0]
    sz = torch.empty(N, 2, dtype=torch.float32, device=dev)
    sd, zd = T(scales), T(zeros)  # keep alive until the kernel ran (caching allocator reuse)
    call(hip, "llj_w4_scale_zero" if bits == 4 else "llj_w8_scale_zero", sd.data_ptr(), zd.data_ptr(), 0,
         sz.data_ptr(), N, st())
    torch.cuda.synchronize()
    return sz


def rand_w8(rng, N, K):
    qw = rng.integers(0, 256, size=(N, K), dtype=np.uint8)
    scales = rng.uniform(0.5, 1.5, size=(N, 1)).astype(np.float32) * np.float32(0.02 / 127)
    zeros = rng.integers(0, 256, size=(N, 1)).astype(np.float32)
    return qw, scales, zeros


def repack8(hip, qw):
    N, K = qw.shape
    ref = T(qw.T.copy())  # physical (K, N) row-major = the reference's column-major bits=8 buffer
    out = torch.empty(N * K, dtype=torch.uint8, device=dev)
    call(hip, "llj_w8_repack", ref.data_ptr(), out.data_ptr(), N, K, st())
    torch.cuda.synchronize()
    return out


def rand_w4g(rng, N, K, g):
    G = (K + g - 1) // g
    qw = rng.integers(0, 256, size=(N, K // 2), dtype=np.uint8)
    scales = rng.uniform(0.5, 1.5, size=(N, G)).astype(np.float32) * np.float32(0.02 / 7)
    zeros = rng.integers(0, 16, size=(N, G)).astype(np.float32)
    return qw, scales, zeros


def sz_grouped(hip, scales, zeros):
    """(scale, 128 + zero) pairs of a grouped int4 weight, group-major (G, N) (wfmt 4)."""
    return sz_of(hip, np.ascontiguousarray(scales.T).reshape(-1, 1), np.ascontiguousarray(zeros.T).reshape(-1, 1))


W4G_128 = 4 | (1 << 8)  # wfmt of grouped int4 with tile_cols = 128


def quant_operands(hip, rng, wfmt, N, K):
    """(reference fp32 weight (N, K), device weight operand, device sz) for wfmt 0 / 1 / 3 and
    grouped int4 (wfmt 4 | (g / 128) << 8)."""
    if wfmt & 0xFF == 4:
        g = 128 * (wfmt >> 8)
        qw, sc, z = rand_w4g(rng, N, K, g)
        return O.colblock_get_weight(qw, sc, z, 4, tile_cols=g), repack(hip, qw), sz_grouped(hip, sc, z)
    if wfmt & ~_hip.WF_ZINT == 0:  # int4 W4P (integral zeros: LLJ_WF_ZINT may be set)
        qw, sc, z = rand_w4(rng, N, K)
        return O.colblock_get_weight(qw, sc, z, 4), repack(hip, qw), sz_of(hip, sc, z)
    if wfmt == 3:
        qw, sc, z = rand_w8(rng, N, K)
        return O.colblock_get_weight(qw, sc, z, 8), repack8(hip, qw), sz_of(hip, sc, z, 8)
    W = bf16(rng.standard_normal((N, K)) / np.sqrt(K))
    return W, T(W, torch.bfloat16), None


@pytest.mark.parametrize("N,K", [(16, 128), (160, 384), (48, 1024)])
def test_w4_repack_layout_and_roundtrip(hip, N, K):
    rng = np.random.default_rng(N + K)
    qw = rng.integers(0, 256, size=(N, K // 2), dtype=np.uint8)
    packed = repack(hip, qw)
    np.testing.assert_array_equal(packed.cpu().numpy(), w4p_pack_np(qw))
    back = torch.empty(K // 2, N, dtype=torch.uint8, device=dev)
    call(hip, "llj_w4_unpack", packed.data_ptr(), back.data_ptr(), N, K, st())
    np.testing.assert_array_equal(back.cpu().numpy().T, qw)


def _linear(hip, wfmt, x, W, sz, N, K, bias=None):
    M = x.shape[0]
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_linear", wfmt, x.data_ptr(), x.stride(0), W.data_ptr(), None if sz is None else sz.data_ptr(),
         None if bias is None else bias.data_ptr(), out.data_ptr(), N, M, N, K, None, 0, None, st())
    torch.cuda.synchronize()
    return out.float().cpu().numpy()


@pytest.mark.parametrize("g,M,N,K", [(g, M, 64, 640) for g in (128, 256, 512) for M in (1, 4, 8, 16)]
                         + [(128, 1, 4096, 4096), (128, 8, 4096, 4096), (256, 1, 4096, 11008), (128, 8, 11008, 4096)])
def test_w4_grouped_linear_shapes(hip, g, M, N, K):
    """Grouped int4 (tile_cols = g: 1, 2 and 4 chunks per group; K = 640 / 11008 leave a ragged last
    group) against the oracle's get_weight (quantization.py:390-409) at decode and 7B shapes."""
    rng = np.random.default_rng(g + M + N + K)
    qw, sc, z = rand_w4g(rng, N, K, g)
    Wref = O.colblock_get_weight(qw, sc, z, 4, tile_cols=g)
    x = bf16(rng.standard_normal((M, K)))
    got = _linear(hip, 4 | ((g // 128) << 8), T(x, torch.bfloat16), repack(hip, qw), sz_grouped(hip, sc, z), N, K)
    assert_bf16_close(got, x.astype(np.float64) @ Wref.T.astype(np.float64), f"w4g g={g}")


def test_w4_grouped_rejects_bad_group(hip):
    """wfmt 4 needs a group size of at least one 128-deep chunk (EINVAL otherwise)."""
    N, K = 32, 256
    x = torch.zeros(1, K, dtype=torch.bfloat16, device=dev)
    w = torch.zeros(N * K // 2, dtype=torch.uint8, device=dev)
    sz = torch.zeros(2 * N, 2, dtype=torch.float32, device=dev)
    out = torch.empty(1, N, dtype=torch.bfloat16, device=dev)
    rc = hip.llj_linear(4, x.data_ptr(), K, w.data_ptr(), sz.data_ptr(), None, out.data_ptr(), N, 1, N, K, None, 0,
                        None, st())
    assert rc == 1000


def test_w4_linear_reference_fixture(hip, golden):
    """The reference's own ColBlockQuantizedLinear buffers (N=160, K=384) and inputs."""
    g = golden("colblock")
    qw, sc, z = g["b4_qw"], g["b4_scales"], g["b4_zeros"]
    N, K = qw.shape[0], qw.shape[1] * 2
    Wp, sz = repack(hip, qw), sz_of(hip, sc, z)
    for M in (1, 3, 8):
        xb = bf16(g[f"b4_x{M}"])
        got = _linear(hip, 0, T(xb, torch.bfloat16), Wp, sz, N, K)
        assert_bf16_close(got, O.qlinear_4bit(xb, qw, sc, z), f"int4 M={M}")
        # and against the reference's fp32 output on the unrounded input
        assert_bf16_close(got, g[f"b4_y{M}"], f"int4 vs reference M={M}", rel=3e-2, abs_frac=1e-2)


@pytest.mark.parametrize("M", [1, 2, 5, 8, 13, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (256, 11008), (2000 * 16, 128)])
def test_w4_linear_shapes(hip, M, N, K):
    rng = np.random.default_rng(M * 7 + N + K)
    qw, sc, z = rand_w4(rng, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    got = _linear(hip, 0, T(x, torch.bfloat16), repack(hip, qw), sz_of(hip, sc, z), N, K)
    assert_bf16_close(got, O.qlinear_4bit(x, qw, sc, z), f"int4 M={M} N={N} K={K}")


@pytest.mark.parametrize("N,K", [(16, 128), (160, 384), (48, 1024)])
def test_w8_repack_layout(hip, N, K):
    rng = np.random.default_rng(3 * N + K)
    qw = rng.integers(0, 256, size=(N, K), dtype=np.uint8)
    packed = repack8(hip, qw)
    np.testing.assert_array_equal(packed.cpu().numpy(), w8p_pack_np(qw))
    back = torch.empty(K, N, dtype=torch.uint8, device=dev)
    call(hip, "llj_w8_unpack", packed.data_ptr(), back.data_ptr(), N, K, st())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(back.cpu().numpy().T, qw)


def test_w8_linear_reference_fixture(hip, golden):
    """gptq.int8: the reference's ColBlockQuantizedLinear(bits=8) buffers (N=160, K=384), its fp32
    forward on the same inputs, and its bf16 path (get_weight(bf16) + F.linear, quantization.py
    419-421, the reference's only bits=8 forward)."""
    g = golden("colblock")
    qw, sc, z = g["b8_qw"], g["b8_scales"], g["b8_zeros"]
    N, K = qw.shape
    Wp, sz = repack8(hip, qw), sz_of(hip, sc, z, 8)
    Wd = O.colblock_get_weight(qw, sc, z, 8)
    for M in (1, 3, 8):
        xb = bf16(g[f"b8_x{M}"])
        got = _linear(hip, 3, T(xb, torch.bfloat16), Wp, sz, N, K)
        assert_bf16_close(got, xb @ Wd.T, f"int8 M={M}")
        assert_bf16_close(got, g[f"b8_y{M}"], f"int8 vs reference fp32 M={M}", rel=3e-2, abs_frac=1e-2)
        assert_bf16_close(got, g[f"b8_ybf16_{M}"], f"int8 vs reference bf16 M={M}", rel=3e-2, abs_frac=1e-2)


@pytest.mark.parametrize("M", [1, 2, 8, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (256, 11008)])
def test_w8_linear_shapes(hip, M, N, K):
    rng = np.random.default_rng(M * 5 + N + K)
    Wref, Wd, sz = quant_operands(hip, rng, 3, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    got = _linear(hip, 3, T(x, torch.bfloat16), Wd, sz, N, K)
    assert_bf16_close(got, x @ Wref.T, f"int8 (gptq) M={M} N={N} K={K}")


@pytest.mark.parametrize("M", [1, 4, 8, 16])
@pytest.mark.parametrize("N,K", [(512, 4096), (64, 11008)])
def test_bf16_linear(hip, M, N, K):
    rng = np.random.default_rng(M + N)
    W = bf16(rng.standard_normal((N, K)) / np.sqrt(K))
    x = bf16(rng.standard_normal((M, K)))
    bias = bf16(rng.standard_normal(N))
    got = _linear(hip, 1, T(x, torch.bfloat16), T(W, torch.bfloat16), None, N, K, T(bias, torch.bfloat16))
    assert_bf16_close(got, x @ W.T + bias, f"bf16 M={M}")


@pytest.mark.parametrize("outliers", [0, 3, 120, 300, 700])
@pytest.mark.parametrize("M", [1, 8])
def test_int8_linear_vs_restatement(hip, M, outliers):
    """LLM.int8() against the oracle's restatement (bitsandbytes absent: parity unpinned). At K 4096
    the side product runs inside the weight stream from the prep's aval table (3 columns: within
    the entries prefetched per chunk; 120: past them, ~4 per chunk); 300 outlier columns (about what
    the synthetic 7B down projection sees at bs=8, K 11008) run it after the stream from the LDS
    stash of CB bytes; 700 (> kStashCols = 512) also the global-read tail."""
    rng = np.random.default_rng(M + 100 * outliers)
    N, K = (256, 4096) if outliers <= 120 else (256, 11008)
    W = bf16(rng.standard_normal((N, K)) * 0.02)
    x = rng.standard_normal((M, K)).astype(np.float32)
    if outliers:
        cols = [17, 1000, 4000] if outliers == 3 else rng.choice(K, outliers, replace=False)
        x[:, cols] *= 25.0
    x = bf16(x)
    Wd = T(W, torch.bfloat16)
    cb = torch.empty(N, K, dtype=torch.int8, device=dev)
    scb = torch.empty(N, dtype=torch.float32, device=dev)
    call(hip, "llj_i8_quant_weight", Wd.data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st())
    cb_ref, scb_ref = O.int8_quantize_weight(W)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cb.cpu().numpy(), cb_ref)
    np.testing.assert_allclose(scb.cpu().numpy(), scb_ref, rtol=0, atol=0)
    # the GEMV reads CB in the I8P tiling; the round trip restores it byte for byte
    cbt = torch.empty_like(cb)
    call(hip, "llj_i8_repack", cb.data_ptr(), cbt.data_ptr(), N, K, st())
    back = torch.empty_like(cb)
    call(hip, "llj_i8_unpack", cbt.data_ptr(), back.data_ptr(), N, K, st())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(back.cpu().numpy(), cb_ref)
    tiles = cbt.cpu().numpy().reshape(N // 16, K // 128, 2, 4, 16, 16)  # (nt, c, t, grp, row, byte)
    np.testing.assert_array_equal(tiles[1, 2, 1, 3, 5], cb_ref[16 + 5, 256 + 64 + 48:256 + 64 + 64])
    cb = cbt
    xd = T(x, torch.bfloat16)
    ws = torch.empty(hip.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", xd.data_ptr(), K, M, K, 6.0, ws.data_ptr(), st())
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_linear", 2, xd.data_ptr(), K, cb.data_ptr(), scb.data_ptr(), None, out.data_ptr(), N, M, N, K,
         ws.data_ptr(), 0, None, st())
    torch.cuda.synchronize()
    ref = O.int8_linear(x, cb_ref, scb_ref)
    assert_bf16_close(out.float().cpu().numpy(), ref, f"int8 M={M} outliers={outliers}", rel=2e-2)


@pytest.mark.parametrize("C", [256, 4096, 5120])
def test_rmsnorm_kernel(hip, golden, C):
    rng = np.random.default_rng(C)
    x = bf16(rng.standard_normal((5, C)) * 3)
    w = bf16(rng.uniform(0.5, 1.5, C))
    xd, wd = T(x, torch.bfloat16), T(w, torch.bfloat16)
    y = torch.empty_like(xd)
    call(hip, "llj_rmsnorm", xd.data_ptr(), wd.data_ptr(), 1e-5, y.data_ptr(), 5, C, st())
    torch.cuda.synchronize()
    assert_bf16_close(y.float().cpu().numpy(), O.rmsnorm(x, w), f"rmsnorm C={C}")
    if C in (256, 4096):  # the reference's own bf16 RMSNorm output
        g = golden("ops")
        xg = T(g[f"rms_x_{C}"].reshape(-1, C), torch.bfloat16)  # fixture input is fp32: bf16-rounded here
        wg = T(g[f"rms_scale_{C}"], torch.bfloat16)
        yg = torch.empty_like(xg)
        call(hip, "llj_rmsnorm", xg.data_ptr(), wg.data_ptr(), 1e-5, yg.data_ptr(), xg.shape[0], C, st())
        torch.cuda.synchronize()
        ref = g[f"rms_ybf16_{C}"].reshape(-1, C)
        diff = np.abs(yg.float().cpu().numpy() - ref)
        ulp2 = np.abs(ref) * 2.0 ** -6  # <= 2 bf16 ulps (rounding points inside torch's bf16 mean differ)
        assert (diff <= ulp2 + 1e-6).all(), f"max diff {diff.max()}"


def _attn_oracle(q, kc, vc, pos, S, T_, nh, hs):
    """numpy attention over the ring cache for rows m = b*T + t at positions pos[t]."""
    M = q.shape[0]
    y = np.zeros_like(q)
    for m in range(M):
        b, t = divmod(m, T_)
        p = int(pos[t])
        slots = np.arange(p + 1) if p < S else np.arange(S)
        for h in range(nh):
            qq = q[m, h * hs:(h + 1) * hs]
            K = kc[b, h, slots]
            V = vc[b, h, slots]
            s = K @ qq / np.sqrt(hs)
            e = np.exp(s - s.max())
            y[m, h * hs:(h + 1) * hs] = (e / e.sum()) @ V
    return y


@pytest.mark.parametrize("hs,nh,B,T_,S,p0", [(128, 4, 1, 1, 144, 80), (128, 3, 8, 1, 144, 143), (64, 4, 2, 5, 16, 0),
                                            (128, 2, 1, 1, 10, 37), (128, 2, 2, 1, 2048, 2000), (128, 32, 1, 1, 256, 90),
                                            (128, 8, 1, 1, 256, 40)])
@pytest.mark.parametrize("spec", ["half", "full", "batch"])
def test_attention(hip, hs, nh, B, T_, S, p0, spec):
    """Decode attention against the oracle; keys loaded before the position is known: a half or a
    whole pass at small grids, or (batch) the half pass at every grid size."""
    from lit_llama import _hip

    with option(hip, _hip.OPT_ATT_SPEC_FULL, 1 if spec == "full" else 0), \
            option(hip, _hip.OPT_ATT_SPEC_BATCH, 1 if spec == "batch" else 0):
        _attention_case(hip, hs, nh, B, T_, S, p0)


def _attention_case(hip, hs, nh, B, T_, S, p0):
    rng = np.random.default_rng(hs + S + p0)
    C = nh * hs
    kc = bf16(rng.standard_normal((B, nh, S, hs)))
    vc = bf16(rng.standard_normal((B, nh, S, hs)))
    q = bf16(rng.standard_normal((B * T_, C)) * 2)
    pos = np.arange(p0, p0 + T_, dtype=np.int32)
    y = torch.empty(B * T_, C, dtype=torch.bfloat16, device=dev)
    qd, kd, vd, pd = T(q, torch.bfloat16), T(kc, torch.bfloat16), T(vc, torch.bfloat16), T(pos)
    call(hip, "llj_attention", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), y.data_ptr(), pd.data_ptr(), B, T_, nh,
         hs, S, st())
    torch.cuda.synchronize()
    assert_bf16_close(y.float().cpu().numpy(), _attn_oracle(q, kc, vc, pos, S, T_, nh, hs), "attention")


def test_argmax_and_advance(hip):
    rng = np.random.default_rng(3)
    V, M = 32000, 8
    L = bf16(rng.standard_normal((M, V)))
    L[2, 7] = L[2, 9] = 50.0  # exact tie: lowest index wins
    Ld = T(L, torch.bfloat16)
    out = torch.empty(M, dtype=torch.int32, device=dev)
    toks = torch.zeros(M, 12, dtype=torch.int32, device=dev)
    pos = torch.tensor([4], dtype=torch.int32, device=dev)
    call(hip, "llj_argmax", Ld.data_ptr(), V, M, V, out.data_ptr(), toks.data_ptr(), 12, pos.data_ptr(), st())
    torch.cuda.synchronize()
    exp = L.argmax(-1)
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    np.testing.assert_array_equal(toks[:, 5].cpu().numpy(), exp)
    assert int(out[2]) == 7


def test_embedding_and_pos_inc(hip):
    rng = np.random.default_rng(4)
    wte = bf16(rng.standard_normal((1000, 256)))
    idx = np.array([5, 999, 0], np.int32)
    out = torch.empty(3, 256, dtype=torch.bfloat16, device=dev)
    pos = torch.tensor([7], dtype=torch.int32, device=dev)
    idd, wd = T(idx), T(wte, torch.bfloat16)
    call(hip, "llj_embedding", idd.data_ptr(), wd.data_ptr(), out.data_ptr(), 3, 256, pos.data_ptr(), st())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.float().cpu().numpy(), wte[idx])
    assert int(pos) == 8


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128])
@pytest.mark.parametrize("B,T_", [(1, 1), (8, 1), (2, 5)])
def test_fused_qkv_rope_kv(hip, wfmt, B, T_):
    rng = np.random.default_rng(wfmt * 10 + B + T_)
    nh, hs = 4, 64
    C, S = nh * hs, 32
    x = bf16(rng.standard_normal((B * T_, C)))
    g = bf16(rng.uniform(0.5, 1.5, C))
    rope = O.build_rope_cache(128, hs)
    pos = np.arange(3, 3 + T_, dtype=np.int32)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, 3 * C, C)
    q = torch.zeros(B * T_, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(B, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    M = B * T_
    xd, gd, rd, pd = T(x, torch.bfloat16), T(g, torch.bfloat16), T(rope), T(pos)
    for r0 in range(0, M, 8):
        r = min(8, M - r0)
        call(hip, "llj_norm_qkv_rope", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, Wd.data_ptr(),
             None if szd is None else szd.data_ptr(), q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rd.data_ptr(),
             pd.data_ptr(), B, T_, C, nh, S, r0, r, None, None, None, 0, st())
    torch.cuda.synchronize()
    h = O.rmsnorm_bf16(x, g)  # the kernels round where the reference does on bf16 tensors
    qkv = bf16(h @ Wref.T)
    qe = O.apply_rope(qkv[:, :C].reshape(B, T_, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(B, T_, nh, hs), rope[pos])
    ve = qkv[:, 2 * C:].reshape(B, T_, nh, hs)
    assert_bf16_close(q.float().cpu().numpy(), qe, "q")
    kcn, vcn = kc.float().cpu().numpy(), vc.float().cpu().numpy()
    for t in range(T_):
        assert_bf16_close(kcn[:, :, pos[t]], ke[:, t], "k cache")
        assert_bf16_close(vcn[:, :, pos[t]], ve[:, t], "v cache")
    untouched = np.ones(S, bool)
    untouched[pos] = False
    assert not kcn[:, :, untouched].any() and not vcn[:, :, untouched].any()


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128])
def test_fused_swiglu_and_resid(hip, wfmt):
    rng = np.random.default_rng(11 + wfmt)
    M, C, H = 3, 256, 768
    x = bf16(rng.standard_normal((M, C)))
    g = bf16(rng.uniform(0.5, 1.5, C))

    def mk(N, K):
        return quant_operands(hip, rng, wfmt, N, K)

    W1, W1d, s1 = mk(H, C)
    W2, W2d, s2 = mk(H, C)
    Wd_, Wdd, sd = mk(C, H)
    h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    xd, gd = T(x, torch.bfloat16), T(g, torch.bfloat16)
    call(hip, "llj_norm_swiglu", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, W1d.data_ptr(), P(s1), W2d.data_ptr(),
         P(s2), h.data_ptr(), M, H, C, None, 0, None, None, 0, st())
    xr = xd.clone()
    call(hip, "llj_linear_resid", wfmt, h.data_ptr(), H, Wdd.data_ptr(), P(sd), xr.data_ptr(), C, M, C, H, None, 0, None,
         st())
    torch.cuda.synchronize()
    hn = O.rmsnorm_bf16(x, g)
    a1, a2 = bf16(hn @ W1.T), bf16(hn @ W2.T)
    hexp = bf16(bf16(O.silu(a1)) * a2)
    # a1, a2, silu(a1) and the product are each rounded to bf16 on the reference path
    # (model.py:258 on bf16 tensors): a 1-ulp flip of a1 or a2 propagates, so allow 3%
    assert_bf16_close(h.float().cpu().numpy(), hexp, "swiglu", rel=3e-2)
    hg = h.float().cpu().numpy()
    assert_bf16_close(xr.float().cpu().numpy(), x + bf16(hg @ Wd_.T), "resid")


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128])
@pytest.mark.parametrize("M", [2, 8, 13])
def test_norm_statistics_handoff(hip, wfmt, M):
    """Batched decode's RMSNorm hand-off: llj_linear_resid writes, per 16-column tile of the new x,
    the partial sums of its bf16-rounded squares (nstat_out); the norm-fused ops that follow
    (rms_2 + SwiGLU, rms_1 + QKV, ln_f + lm_head) take those partials instead of recomputing the
    sums from x. The partials must add up to the sum of squares of the stored x, and the fused
    ops must give what they give without the hand-off (only the fp32 summation order differs)."""
    rng = np.random.default_rng(300 + 7 * wfmt + M)
    C, H, nh, hs, S, V = 512, 768, 4, 128, 16, 1024
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    x0 = bf16(rng.standard_normal((M, C)))
    hin = bf16(rng.standard_normal((M, H)))
    g = bf16(rng.uniform(0.5, 1.5, C))
    Wd_, Wdd, sd = quant_operands(hip, rng, wfmt, C, H)
    npart = C // 16
    nst = torch.full((npart * 16,), float("nan"), dtype=torch.float32, device=dev)
    xd, hd, gd = T(x0, torch.bfloat16), T(hin, torch.bfloat16), T(g, torch.bfloat16)
    for r0 in range(0, M, 16):
        r = min(16, M - r0)
        call(hip, "llj_linear_resid", wfmt, hd[r0].data_ptr(), H, Wdd.data_ptr(), P(sd), xd[r0].data_ptr(), C, r, C,
             H, None, 0, nst[r0:].data_ptr(), st())
    torch.cuda.synchronize()
    xn = xd.float().cpu().numpy()
    part = nst.cpu().numpy().reshape(npart, 16)[:, :M]
    assert np.isfinite(part).all()
    sq = bf16(xn * xn).astype(np.float64)  # x * x in bf16 (model.py:281)
    np.testing.assert_allclose(part.sum(0), sq.sum(1), rtol=1e-5)
    for t in range(npart):  # every tile's partial is its own 16 columns
        np.testing.assert_allclose(part[t], sq[:, 16 * t:16 * t + 16].sum(1), rtol=1e-5, atol=1e-6)

    def both(run):
        a = run(None)
        b = run(nst)
        torch.cuda.synchronize()
        return a.float().cpu().numpy(), b.float().cpu().numpy()

    W1, W1d, s1 = quant_operands(hip, rng, wfmt, H, C)
    W2, W2d, s2 = quant_operands(hip, rng, wfmt, H, C)

    def swiglu(ns):
        h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
        for r0 in range(0, M, 8):
            r = min(8, M - r0)
            call(hip, "llj_norm_swiglu", wfmt, xd[r0].data_ptr(), gd.data_ptr(), 1e-5, W1d.data_ptr(), P(s1),
                 W2d.data_ptr(), P(s2), h[r0].data_ptr(), r, H, C, None, 0, None,
                 None if ns is None else ns[r0:].data_ptr(), npart, st())
        return h

    a, b = both(swiglu)
    hn = bf16(O.rmsnorm(xn, g))
    hexp = bf16(bf16(O.silu(bf16(hn @ W1.T))) * bf16(hn @ W2.T))
    assert_bf16_close(a, hexp, "swiglu", rel=3e-2)
    assert_bf16_close(b, hexp, "swiglu hand-off", rel=3e-2)
    assert np.mean(a == b) > 0.999, np.mean(a == b)
    Wq, Wqd, sqd = quant_operands(hip, rng, wfmt, 3 * C, C)
    rope, pos = T(O.build_rope_cache(32, hs)), T(np.array([5], np.int32))

    def qkv(ns):
        q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
        kc = torch.zeros(M, nh, S, hs, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        for r0 in range(0, M, 8):
            r = min(8, M - r0)
            call(hip, "llj_norm_qkv_rope", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, Wqd.data_ptr(), P(sqd),
                 q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rope.data_ptr(), pos.data_ptr(), M, 1, C, nh, S, r0, r,
                 None, None, P(ns), npart, st())
        return torch.cat([q.reshape(M, -1), kc.reshape(M, -1), vc.reshape(M, -1)], 1)

    a, b = both(qkv)
    assert np.mean(a == b) > 0.999, np.mean(a == b)
    Wh, Whd, shd = quant_operands(hip, rng, wfmt, V, C)

    def head(ns):
        lg = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        for r0 in range(0, M, 8):
            r = min(8, M - r0)
            call(hip, "llj_norm_linear", wfmt, xd[r0].data_ptr(), gd.data_ptr(), 1e-5, Whd.data_ptr(), P(shd),
                 lg[r0].data_ptr(), V, r, V, C, None, 0, None, None if ns is None else ns[r0:].data_ptr(), npart,
                 st())
        return lg

    a, b = both(head)
    assert np.mean(a == b) > 0.999, np.mean(a == b)
    # the hand-off is refused where it is not defined: int8, more rows than the partial stride
    bad = torch.zeros(64, dtype=torch.bfloat16, device=dev)
    assert hip.llj_norm_swiglu(wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, W1d.data_ptr(), P(s1),
                               W2d.data_ptr(), P(s2), bad.data_ptr(), M, H, C, None, 0, None, nst.data_ptr(), 10000,
                               st()) == 1000


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128])
@pytest.mark.parametrize("M", [2, 5, 8])
def test_streamed_a_equals_lds_image_forms(hip, wfmt, M):
    """Batched rows (2..8) stream their A rows per K chunk (gemv_impl.h AM_STREAM / AM_SNORM,
    llj_set_stream_a(1), the default) instead of staging one LDS image per workgroup
    (llj_set_stream_a(0)). The MFMA operands are the same bf16 values, so the plain ops agree
    bitwise where both take the same row-sum route (bf16; the 8-wave long-K residual, whose image
    does not fit the LDS), and elsewhere up to the int4 offset's fp32 row sums (MFMA against a ones
    fragment vs VALU); the fused-norm ops normalize from the producer's partials (nstat) in both.
    All of them match the oracle at 7B widths (K 4096 / 11008, 768 / 688 / 256-tile grids)."""
    rng = np.random.default_rng(700 + 7 * (wfmt & 0xFF) + M)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    C, nh, hs, H, S = 4096, 32, 128, 11008, 64
    x0 = bf16(rng.standard_normal((M, C)))
    hin = bf16(rng.standard_normal((M, H)))
    yin = bf16(rng.standard_normal((M, C)))
    g = bf16(rng.uniform(0.5, 1.5, C))
    xd, hd, yd, gd = T(x0, torch.bfloat16), T(hin, torch.bfloat16), T(yin, torch.bfloat16), T(g, torch.bfloat16)
    Wq, Wqd, sq = quant_operands(hip, rng, wfmt, 3 * C, C)
    Wo, Wod, so = quant_operands(hip, rng, wfmt, C, C)
    W1, W1d, s1 = quant_operands(hip, rng, wfmt, H, C)
    W2, W2d, s2 = quant_operands(hip, rng, wfmt, H, C)
    Wd_, Wdd, sd = quant_operands(hip, rng, wfmt, C, H)
    rope, pos = T(O.build_rope_cache(128, hs)), T(np.array([41], np.int32))
    npart = C // 16

    def run(stream):
        old = hip.llj_set_stream_a(stream)
        try:
            nst = torch.full((npart * 16,), float("nan"), dtype=torch.float32, device=dev)
            x = xd.clone()
            call(hip, "llj_linear_resid", wfmt, hd.data_ptr(), H, Wdd.data_ptr(), P(sd), x.data_ptr(), C, M, C, H, None,
                 0, nst.data_ptr(), st())  # producer: mlp.c_proj + the next norm's partials
            q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
            kc = torch.zeros(M, nh, S, hs, dtype=torch.bfloat16, device=dev)
            vc = torch.zeros_like(kc)
            call(hip, "llj_norm_qkv_rope", wfmt, x.data_ptr(), gd.data_ptr(), 1e-5, Wqd.data_ptr(), P(sq), q.data_ptr(),
                 kc.data_ptr(), vc.data_ptr(), rope.data_ptr(), pos.data_ptr(), M, 1, C, nh, S, 0, M, None, None,
                 nst.data_ptr(), npart, st())
            x2 = x.clone()
            nst2 = torch.full_like(nst, float("nan"))
            call(hip, "llj_linear_resid", wfmt, yd.data_ptr(), C, Wod.data_ptr(), P(so), x2.data_ptr(), C, M, C, C, None,
                 0, nst2.data_ptr(), st())  # attn.c_proj (K = C)
            h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
            call(hip, "llj_norm_swiglu", wfmt, x2.data_ptr(), gd.data_ptr(), 1e-5, W1d.data_ptr(), P(s1), W2d.data_ptr(),
                 P(s2), h.data_ptr(), M, H, C, None, 0, None, nst2.data_ptr(), npart, st())
            lin = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
            call(hip, "llj_linear", wfmt, yd.data_ptr(), C, Wod.data_ptr(), P(so), None, lin.data_ptr(), C, M, C, C,
                 None, 0, None, st())
            torch.cuda.synchronize()
        finally:
            hip.llj_set_stream_a(old)
        return dict(x=x, q=q, k=kc[:, :, 41], v=vc[:, :, 41], x2=x2, h=h, lin=lin)

    img, strm = run(0), run(1)
    for name in img:
        a, b = img[name].float().cpu().numpy(), strm[name].float().cpu().numpy()
        if wfmt in (1, W4G_128) or (name == "x" and M >= 5):  # same row-sum route (or none)
            assert np.array_equal(a, b), name
        else:  # the offset term (128 + z) * sum_k A cancels most of sum_k A (128 + q): an fp32 ulp of
            # the row sum moves the bf16 output by one ulp now and then (both routes checked below)
            assert np.mean(a == b) > 0.9, (name, np.mean(a == b))
            assert_bf16_close(b, a, name)
    # the streamed forms against the oracle
    xs = strm["x"].float().cpu().numpy()
    assert_bf16_close(xs, x0 + bf16(hin @ Wd_.T), "mlp.c_proj resid")
    hn = O.rmsnorm_bf16(xs, g)
    qkv = bf16(hn @ Wq.T)
    assert_bf16_close(strm["q"].float().cpu().numpy(),
                      O.apply_rope(qkv[:, :C].reshape(M, 1, nh, hs), O.build_rope_cache(128, hs)[[41]]).reshape(M, C), "q")
    assert_bf16_close(strm["v"].float().cpu().numpy().reshape(M, C), qkv[:, 2 * C:], "v")
    x2 = strm["x2"].float().cpu().numpy()
    assert_bf16_close(x2, xs + bf16(yin @ Wo.T), "attn.c_proj resid")
    hn2 = O.rmsnorm_bf16(x2, g)
    hexp = bf16(bf16(O.silu(bf16(hn2 @ W1.T))) * bf16(hn2 @ W2.T))
    assert_bf16_close(strm["h"].float().cpu().numpy(), hexp, "swiglu", rel=3e-2)
    assert_bf16_close(strm["lin"].float().cpu().numpy(), yin @ Wo.T, "linear")


def test_rmsnorm_rows_rowsum_and_int4_rowsum_operand(hip, golden):
    """llj_rmsnorm_rows: same normalized rows as llj_rmsnorm plus fp32 row sums; an int4 GEMV
    fed those sums (rowsum operand) equals the one that reduces them in-kernel."""
    rng = np.random.default_rng(5)
    M, C, N = 5, 512, 256
    x = T(bf16(rng.standard_normal((M, C))), torch.bfloat16)
    g = T(bf16(rng.uniform(0.5, 1.5, C)), torch.bfloat16)
    y1 = torch.empty_like(x)
    y2 = torch.empty_like(x)
    rs = torch.empty(M, dtype=torch.float32, device=dev)
    call(hip, "llj_rmsnorm", x.data_ptr(), g.data_ptr(), 1e-5, y1.data_ptr(), M, C, st())
    call(hip, "llj_rmsnorm_rows", x.data_ptr(), g.data_ptr(), 1e-5, y2.data_ptr(), rs.data_ptr(), M, C, st())
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    np.testing.assert_allclose(rs.cpu().numpy(), y2.float().sum(1).cpu().numpy(), rtol=1e-5, atol=1e-3)
    qw, sc, z = rand_w4(rng, N, C)
    Wd, szd = repack(hip, qw), sz_of(hip, sc, z)
    outs = []
    for r in (None, rs):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        call(hip, "llj_linear", 0, y2.data_ptr(), C, Wd.data_ptr(), szd.data_ptr(), None, out.data_ptr(), N, M, N, C,
             None, 0, None if r is None else r.data_ptr(), st())
        outs.append(out)
    torch.cuda.synchronize()
    ref = bf16(y2.float().cpu().numpy() @ O.colblock_get_weight(qw, sc, z, 4).T)
    for o in outs:
        assert_bf16_close(o.float().cpu().numpy(), ref, "int4 with/without rowsum")


@pytest.mark.parametrize("wfmt", [0, 3])
@pytest.mark.parametrize("M", [7, 8])
def test_multi_tile_workgroups_equal_single_tile(hip, wfmt, M):
    """Several 16-column tiles per workgroup (7B / 13B shapes: QKV 768 tiles, SwiGLU 688 with a
    partial last workgroup, lm_head 2000, 13B mlp.c_proj 320 tiles at 8 waves) give bitwise
    the results of one tile per workgroup (llj_set_tpw_max(1)), and match the oracle."""
    rng = np.random.default_rng(100 + M + wfmt)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    C, nh, H, V = 4096, 32, 11008, 32000
    x = bf16(rng.standard_normal((M, C)))
    g = bf16(rng.uniform(0.5, 1.5, C))
    xd, gd = T(x, torch.bfloat16), T(g, torch.bfloat16)
    _, Wqd, sq = quant_operands(hip, rng, wfmt, 3 * C, C)
    W1, W1d, s1 = quant_operands(hip, rng, wfmt, H, C)
    W2, W2d, s2 = quant_operands(hip, rng, wfmt, H, C)
    Wh, Whd, sh = quant_operands(hip, rng, wfmt, V, C)
    C13, H13 = 5120, 13824
    Wr, Wrd, sr = quant_operands(hip, rng, wfmt, C13, H13)
    hx = bf16(rng.standard_normal((M, H13)))
    hxd = T(hx, torch.bfloat16)
    xr0 = T(bf16(rng.standard_normal((M, C13))), torch.bfloat16)
    rope, pos, S = T(O.build_rope_cache(256, 128)), T(np.array([37], np.int32)), 64

    def run():
        q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
        kc = torch.zeros(M, nh, S, 128, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        call(hip, "llj_norm_qkv_rope", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, Wqd.data_ptr(), P(sq), q.data_ptr(),
             kc.data_ptr(), vc.data_ptr(), rope.data_ptr(), pos.data_ptr(), M, 1, C, nh, S, 0, M, None, None, None, 0, st())
        h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
        call(hip, "llj_norm_swiglu", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, W1d.data_ptr(), P(s1), W2d.data_ptr(),
             P(s2), h.data_ptr(), M, H, C, None, 0, None, None, 0, st())
        lg = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        call(hip, "llj_norm_linear", wfmt, xd.data_ptr(), gd.data_ptr(), 1e-5, Whd.data_ptr(), P(sh), lg.data_ptr(),
             V, M, V, C, None, 0, None, None, 0, st())
        xr = xr0.clone()
        call(hip, "llj_linear_resid", wfmt, hxd.data_ptr(), H13, Wrd.data_ptr(), P(sr), xr.data_ptr(), C13, M, C13,
             H13, None, 0, None, st())
        torch.cuda.synchronize()
        return q, kc, vc, h, lg, xr

    old = hip.llj_set_tpw_max(1)
    try:
        one = run()
    finally:
        hip.llj_set_tpw_max(old)
    multi = run()
    for name, a, b in zip(("q", "k cache", "v cache", "swiglu", "lm_head", "resid"), one, multi):
        assert torch.equal(a, b), name
    hn = bf16(O.rmsnorm(x, g))
    hexp = bf16(bf16(O.silu(bf16(hn @ W1.T))) * bf16(hn @ W2.T))
    assert_bf16_close(multi[3].float().cpu().numpy(), hexp, "swiglu", rel=3e-2)
    assert_bf16_close(multi[4].float().cpu().numpy(), hn @ Wh.T, "lm_head")
    assert_bf16_close(multi[5].float().cpu().numpy(), xr0.float().cpu().numpy() + bf16(hx @ Wr.T), "resid 13B")


@pytest.mark.parametrize("M,K", [(1, 4096), (8, 4096), (13, 4096), (3, 256), (8, 5120), (16, 5120), (20, 4096), (5, 11008)])
def test_i8_norm_stats_equals_separate_launches(hip, M, K):
    """llj_i8_norm_stats (one launch for M <= 8, K <= 4096; RMSNorm + pass 1, then the row
    quantization up to 16 rows; the two ops beyond) is bit-identical to llj_rmsnorm followed by
    llj_i8_stats (itself one launch for M <= 8, K <= 4096, else two passes): the normalized rows
    and every byte of the statistics workspace, which also matches the numpy restatement."""
    rng = np.random.default_rng(M * 7 + K)
    x = bf16(rng.standard_normal((M, K)))
    x[:, rng.choice(K, 5, replace=False)] *= 40.0  # outlier columns after the norm
    g = bf16(rng.uniform(0.5, 1.5, K))
    xd, gd = T(x, torch.bfloat16), T(g, torch.bfloat16)
    nb = hip.llj_i8_ws_bytes(M, K)
    ws1 = torch.zeros(nb, dtype=torch.uint8, device=dev)
    ws2 = torch.zeros(nb, dtype=torch.uint8, device=dev)
    xn1 = torch.zeros(M, K, dtype=torch.bfloat16, device=dev)
    xn2 = torch.zeros(M, K, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_rmsnorm", xd.data_ptr(), gd.data_ptr(), 1e-5, xn1.data_ptr(), M, K, st())
    call(hip, "llj_i8_stats", xn1.data_ptr(), K, M, K, 6.0, ws1.data_ptr(), st())
    call(hip, "llj_i8_norm_stats", xd.data_ptr(), gd.data_ptr(), 1e-5, xn2.data_ptr(), M, K, 6.0, ws2.data_ptr(), st())
    torch.cuda.synchronize()
    assert torch.equal(xn1.view(torch.int16), xn2.view(torch.int16))
    assert torch.equal(ws1, ws2)
    assert (np.abs(xn1.float().cpu().numpy()) >= 6.0).any()  # the case has outlier columns
    _check_i8_ws(ws1.cpu().numpy(), xn1.float().cpu().numpy(), M, K)


def _check_i8_ws(ws, a, M, K, thr=6.0):
    """The statistics workspace (csrc/i8ws.h) against a numpy restatement of the LLM.int8() rules
    (oracle/llama_np.py int8_linear): A16 = A.half(); outlier columns = any row |A16| >= thr, listed
    ascending per k-block; SCA = row max of the other elements; aq = round(A16 * 127 / SCA),
    outlier columns 0; part = the per-(k-block, row) maxima."""
    nsb = 32
    kb = ((K + nsb - 1) // nsb + 31) & ~31
    a16 = np.abs(a.astype(np.float16).astype(np.float32))
    out = a16 >= thr
    flag = out.any(0)
    small = np.where(out, 0.0, a16)
    al = lambda x: (x + 15) & ~15  # noqa: E731
    o_aq = 16  # the quantized rows first (csrc/i8ws.h), then the statistics
    o_part = al(o_aq + M * K)
    o_cnt = o_part + 4 * nsb * M
    o_list = o_cnt + 4 * nsb
    o_sca = o_list + 4 * nsb * kb
    o_flag = al(o_sca + 4 * M)
    hdr = ws[:16].view(np.int32)
    assert list(hdr) == [M, K, nsb, kb]
    part = ws[o_part:o_cnt].view(np.float32).reshape(nsb, M)
    cnt = ws[o_cnt:o_list].view(np.int32)
    lst = ws[o_list:o_sca].view(np.int32).reshape(nsb, kb)
    sca = ws[o_sca:o_sca + 4 * M].view(np.float32)
    np.testing.assert_array_equal(ws[o_flag:o_flag + K], flag.astype(np.uint8))
    np.testing.assert_array_equal(sca, small.max(1))
    for b in range(nsb):
        cols = np.nonzero(flag[b * kb:(b + 1) * kb])[0] + b * kb
        assert cnt[b] == len(cols)
        np.testing.assert_array_equal(lst[b, :len(cols)], cols)
        blk = small[:, b * kb:(b + 1) * kb]
        np.testing.assert_array_equal(part[b], blk.max(1) if blk.size else np.zeros(M, np.float32))
    inv = np.where(sca > 0, np.float32(127) / sca, np.float32(0)).astype(np.float32)
    q = np.clip(np.rint(a.astype(np.float16).astype(np.float32) * inv[:, None]), -127, 127)
    q[:, flag] = 0
    np.testing.assert_array_equal(ws[o_aq:o_aq + M * K].view(np.int8).reshape(M, K), q.astype(np.int8))


@pytest.mark.parametrize("wfmt", [0, 3, W4G_128])
def test_long_k_residual_eight_waves_m1(hip, wfmt):
    """mlp.c_proj at 7B (K = 11008 >= 8192: 8-wave workgroups, M = 1 register prologue): every
    wave's A row sum lands in the LDS tail (the int4 / int8 offset removal needs all eight)."""
    rng = np.random.default_rng(7 + wfmt)
    N, K = 4096, 11008
    W, Wd, szd = quant_operands(hip, rng, wfmt, N, K)
    h = bf16(rng.standard_normal((1, K)))
    x0 = bf16(rng.standard_normal((1, N)))
    xd = T(x0, torch.bfloat16)
    call(hip, "llj_linear_resid", wfmt, T(h, torch.bfloat16).data_ptr(), K, Wd.data_ptr(), szd.data_ptr(),
         xd.data_ptr(), N, 1, N, K, None, 0, None, st())
    torch.cuda.synchronize()
    assert_bf16_close(xd.float().cpu().numpy(), x0 + bf16(h @ W.T), "resid K=11008 M=1")


@pytest.mark.parametrize("hs,nh,B,T_,S,p0,nsplit", [(128, 4, 1, 1, 2048, 2000, 16), (128, 3, 2, 1, 2048, 40, 16),
                                                   (64, 4, 2, 5, 600, 300, 5), (128, 2, 1, 1, 512, 900, 4),
                                                   (128, 2, 8, 1, 1024, 1023, 8)])
def test_attention_split_keys(hip, hs, nh, B, T_, S, p0, nsplit):
    """Split-K attention (key ranges per block + in-order merge) against the oracle, incl. empty
    ranges (p0 small), prefill rows (T > 1) and the rolled ring (p0 >= S)."""
    rng = np.random.default_rng(hs + S + p0 + nsplit)
    C = nh * hs
    kc = bf16(rng.standard_normal((B, nh, S, hs)))
    vc = bf16(rng.standard_normal((B, nh, S, hs)))
    q = bf16(rng.standard_normal((B * T_, C)) * 2)
    pos = np.arange(p0, p0 + T_, dtype=np.int32)
    y = torch.empty(B * T_, C, dtype=torch.bfloat16, device=dev)
    ws = torch.empty(hip.llj_attention_ws_bytes(B * T_, nh, hs, nsplit), dtype=torch.uint8, device=dev)
    qd, kd, vd, pd = T(q, torch.bfloat16), T(kc, torch.bfloat16), T(vc, torch.bfloat16), T(pos)
    call(hip, "llj_attention_split", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), y.data_ptr(), pd.data_ptr(), B, T_,
         nh, hs, S, nsplit, ws.data_ptr(), st())
    torch.cuda.synchronize()
    assert_bf16_close(y.float().cpu().numpy(), _attn_oracle(q, kc, vc, pos, S, T_, nh, hs), "split attention")


def _i8_ws_stats(hip, A, M, K):
    """(SCA (M,), outlier flags (K,) bool) of llj_i8_stats's workspace for the rows A (M, K)."""
    from lit_llama import _hip

    ws = torch.empty(hip.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", A.data_ptr(), A.stride(0), M, K, 6.0, ws.data_ptr(), st())
    torch.cuda.synchronize()
    raw = ws.cpu().numpy()
    # i8ws.h layout: header, aq[M][K], part[32][M], cnt[32], list[32][kb], sca[M], flag[K] (16-B aligned)
    kb = ((K + 31) // 32 + 31) & ~31
    o_part = (16 + M * K + 15) & ~15
    o_sca = o_part + 4 * 32 * M + 4 * 32 + 4 * 32 * kb
    o_flag = (o_sca + 4 * M + 15) & ~15
    return raw[o_sca:o_sca + 4 * M].view(np.float32), raw[o_flag:o_flag + K] != 0


def _st_decode(st, M, K):
    """(SCA (M,), outlier flags (K,)) of a hand-off statistics block (i8ws.h: 64 SCA slots of 8 rows
    from word 16, the flag bits from word 16 + 512)."""
    w = st.cpu().numpy().view(np.uint32)
    sca = w[16:16 + 512].view(np.float32).reshape(64, 8).max(0)[:M]
    flags = np.unpackbits(w[528:528 + (K + 31) // 32].view(np.uint8), bitorder="little")[:K] != 0
    return sca, flags


@pytest.mark.parametrize("M", [1, 5, 8])
@pytest.mark.parametrize("regime", ["none", "few", "many"])
def test_int8_statistics_handoff(hip, M, regime):
    """LLM.int8 decode rows without the statistics launches of y and h: llj_attention_i8 and
    llj_i8_swiglu_stats write the row statistics of their outputs (SCA and outlier columns by
    order-independent atomics: bitwise the values llj_i8_stats computes) and zero the other block;
    llj_i8_linear_resid quantizes its bf16 rows per chunk from them and takes the fp16 side product
    from the streamed weights -- the same int8 codes as the workspace path (only the side product's
    fp32 order differs) and the oracle's LLM.int8() result. 7B shapes (C 4096, 32 heads, H 11008)."""
    from lit_llama import _hip

    rng = np.random.default_rng(1300 + 10 * M + len(regime))
    C, nh, H, S = 4096, 32, 11008, 64
    hs = C // nh
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731

    def wq(N, K):
        W = bf16(rng.standard_normal((N, K)) * 0.02)
        Wd = T(W, torch.bfloat16)
        cb = torch.empty(N, K, dtype=torch.int8, device=dev)
        scb = torch.empty(N, dtype=torch.float32, device=dev)
        call(hip, "llj_i8_quant_weight", Wd.data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st())
        cbt = torch.empty_like(cb)
        call(hip, "llj_i8_repack", cb.data_ptr(), cbt.data_ptr(), N, K, st())
        torch.cuda.synchronize()
        return O.int8_quantize_weight(W), cbt, scb

    scale = {"none": 0.5, "few": 1.0, "many": 3.0}[regime]
    # attention over a cache: y rows; v scaled so that y has (regime) outlier columns
    kc = T(bf16(rng.standard_normal((M, nh, S, hs))), torch.bfloat16)
    vv = rng.standard_normal((M, nh, S, hs)).astype(np.float32) * scale
    if regime == "few":
        vv[:, 3, :, 7] = 9.0  # one y column >= 6 in every row
    vc = T(bf16(vv), torch.bfloat16)
    q = T(bf16(rng.standard_normal((M, C))), torch.bfloat16)
    pos = T(np.array([40], np.int32))
    y = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    y_st = torch.full((hip.llj_i8_rowstats_bytes(C) // 4,), 0, dtype=torch.int32, device=dev)
    h_st = torch.full((hip.llj_i8_rowstats_bytes(H) // 4,), 7, dtype=torch.int32, device=dev)  # to be zeroed
    call(hip, "llj_attention_i8", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), y.data_ptr(), pos.data_ptr(), M, 1, nh,
         hs, S, 1, None, y_st.data_ptr(), h_st.data_ptr(), h_st.numel(), 6.0, st())
    torch.cuda.synchronize()
    assert not h_st.any()
    y_ref = torch.empty_like(y)
    call(hip, "llj_attention", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), y_ref.data_ptr(), pos.data_ptr(), M, 1, nh, hs,
         S, st())
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    sca_w, fl_w = _i8_ws_stats(hip, y, M, C)
    sca_s, fl_s = _st_decode(y_st, M, C)
    np.testing.assert_array_equal(sca_s, sca_w)
    np.testing.assert_array_equal(fl_s, fl_w)
    if regime == "few":
        assert fl_s.any()
    # c_proj + residual from y's statistics vs the workspace path and the oracle
    (cbo, scbo), cbod, scbod = wq(C, C)
    x0 = T(bf16(rng.standard_normal((M, C))), torch.bfloat16)
    xa, xb = x0.clone(), x0.clone()
    call(hip, "llj_i8_linear_resid", y.data_ptr(), C, cbod.data_ptr(), scbod.data_ptr(), xa.data_ptr(), C, M, C, C,
         y_st.data_ptr(), st())
    ws = torch.empty(hip.llj_i8_ws_bytes(M, H), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", y.data_ptr(), C, M, C, 6.0, ws.data_ptr(), st())
    call(hip, "llj_linear_resid", 2, y.data_ptr(), C, cbod.data_ptr(), scbod.data_ptr(), xb.data_ptr(), C, M, C, C,
         ws.data_ptr(), 0, None, st())
    torch.cuda.synchronize()
    a, b = xa.float().cpu().numpy(), xb.float().cpu().numpy()
    assert np.mean(a == b) > 0.98, np.mean(a == b)
    if not fl_s.any():  # no outlier columns: identical int8 codes and exact int32 sums -> bitwise equal
        assert np.array_equal(a, b)  # (the per-chunk quantization, quant8_fast, is the statistics launch's)
    yh = y.float().cpu().numpy()
    assert_bf16_close(a, x0.float().cpu().numpy() + bf16(O.int8_linear(yh, cbo, scbo)), f"int8 c_proj M={M}")
    # SwiGLU over normalized rows -> h and its statistics (and y's block zeroed)
    xn = rng.standard_normal((M, C)).astype(np.float32) * scale
    if regime == "few":
        xn[:, [17, 3001]] *= 8.0
    xn = bf16(xn)
    xnd = T(xn, torch.bfloat16)
    n_st = torch.full((hip.llj_i8_rowstats_bytes(C) // 4,), 3, dtype=torch.int32, device=dev)  # rewritten whole
    call(hip, "llj_i8_norm_rowstats", xnd.data_ptr(), None, 1e-5, None, M, C, 6.0, ws.data_ptr(), n_st.data_ptr(), st())
    torch.cuda.synchronize()
    sca_w, fl_w = _i8_ws_stats(hip, xnd, M, C)  # (re-runs llj_i8_stats into ws for the workspace path below)
    sca_s, fl_s = _st_decode(n_st, M, C)
    np.testing.assert_array_equal(sca_s, sca_w)
    np.testing.assert_array_equal(fl_s, fl_w)
    call(hip, "llj_i8_stats", xnd.data_ptr(), C, M, C, 6.0, ws.data_ptr(), st())
    (cb1, scb1), cb1d, scb1d = wq(H, C)
    (cb2, scb2), cb2d, scb2d = wq(H, C)
    # larger fc weights in the "many" regime: h with hundreds of outlier columns (the random weights' own)
    h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    h_ref = torch.empty_like(h)
    h_ws = torch.empty_like(h)  # the same with xn's statistics launch workspace (the model's default)
    h_st2 = torch.zeros_like(h_st)
    call(hip, "llj_i8_swiglu_stats", xnd.data_ptr(), cb1d.data_ptr(), scb1d.data_ptr(), cb2d.data_ptr(), scb2d.data_ptr(),
         h_ws.data_ptr(), M, H, C, ws.data_ptr(), None, h_st2.data_ptr(), None, 0, 6.0, st())
    call(hip, "llj_i8_swiglu_stats", xnd.data_ptr(), cb1d.data_ptr(), scb1d.data_ptr(), cb2d.data_ptr(), scb2d.data_ptr(),
         h.data_ptr(), M, H, C, None, n_st.data_ptr(), h_st.data_ptr(), y_st.data_ptr(), y_st.numel(), 6.0, st())
    call(hip, "llj_norm_swiglu", 2, xnd.data_ptr(), None, 1e-5, cb1d.data_ptr(), scb1d.data_ptr(), cb2d.data_ptr(),
         scb2d.data_ptr(), h_ref.data_ptr(), M, H, C, ws.data_ptr(), 0, None, None, 0, st())
    torch.cuda.synchronize()
    # same int8 codes; the fp16 side product's fp32 order differs (in-stream vs after the stream)
    assert np.mean(h.float().cpu().numpy() == h_ref.float().cpu().numpy()) > 0.98
    assert torch.equal(h_ws, h_ref)  # the workspace form is the LDS-image SwiGLU with statistics added
    for got, want in zip(_st_decode(h_st2, M, H), _i8_ws_stats(hip, h_ws, M, H)):
        np.testing.assert_array_equal(got, want)
    hexp = bf16(bf16(O.silu(bf16(O.int8_linear(xn, cb1, scb1)))) * bf16(O.int8_linear(xn, cb2, scb2)))
    assert_bf16_close(h.float().cpu().numpy(), hexp, f"int8 swiglu (streamed) M={M}", rel=3e-2)
    assert not y_st.any()
    sca_w, fl_w = _i8_ws_stats(hip, h, M, H)  # h's statistics from the streamed SwiGLU's own output
    sca_s, fl_s = _st_decode(h_st, M, H)
    np.testing.assert_array_equal(sca_s, sca_w)
    np.testing.assert_array_equal(fl_s, fl_w)
    print(f"[int8 hand-off] M={M} {regime}: y outlier columns {int(_st_decode(y_st, M, C)[1].sum())}, "
          f"h outlier columns {int(fl_s.sum())}")
    (cbd_, scbd_), cbdd, scbdd = wq(C, H)
    xa, xb = x0.clone(), x0.clone()
    call(hip, "llj_i8_linear_resid", h.data_ptr(), H, cbdd.data_ptr(), scbdd.data_ptr(), xa.data_ptr(), C, M, C, H,
         h_st.data_ptr(), st())
    call(hip, "llj_i8_stats", h.data_ptr(), H, M, H, 6.0, ws.data_ptr(), st())
    call(hip, "llj_linear_resid", 2, h.data_ptr(), H, cbdd.data_ptr(), scbdd.data_ptr(), xb.data_ptr(), C, M, C, H,
         ws.data_ptr(), 0, None, st())
    torch.cuda.synchronize()
    a, b = xa.float().cpu().numpy(), xb.float().cpu().numpy()
    assert np.mean(a == b) > 0.98, np.mean(a == b)
    hh = h.float().cpu().numpy()
    assert_bf16_close(a, x0.float().cpu().numpy() + bf16(O.int8_linear(hh, cbd_, scbd_)), f"int8 mlp.c_proj M={M}")
    # QKV + RoPE + KV write and lm_head-style store on the norm rows' hand-off block (wfmt 2 | ROWSTATS)
    (cbq, scbq), cbqd, scbqd = wq(3 * C, C)
    rope = O.build_rope_cache(128, hs)
    roped = T(rope)
    qo = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kq = torch.zeros(M, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vq = torch.zeros_like(kq)
    call(hip, "llj_norm_qkv_rope", 2 | _hip.WF_I8_ROWSTATS, xnd.data_ptr(), None, 1e-5, cbqd.data_ptr(), scbqd.data_ptr(),
         qo.data_ptr(), kq.data_ptr(), vq.data_ptr(), roped.data_ptr(), pos.data_ptr(), M, 1, C, nh, S, 0, M,
         n_st.data_ptr(), None, None, 0, st())
    lo = torch.empty(M, 3 * C, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_norm_linear", 2 | _hip.WF_I8_ROWSTATS, xnd.data_ptr(), None, 1e-5, cbqd.data_ptr(), scbqd.data_ptr(),
         lo.data_ptr(), 3 * C, M, 3 * C, C, n_st.data_ptr(), 0, None, None, 0, st())
    torch.cuda.synchronize()
    qkv = bf16(O.int8_linear(xn, cbq, scbq))
    assert_bf16_close(lo.float().cpu().numpy(), qkv, f"int8 linear (streamed) M={M}")
    qe = O.apply_rope(qkv[:, :C].reshape(M, 1, nh, hs), rope[[40]]).reshape(M, C)
    assert_bf16_close(qo.float().cpu().numpy(), qe, f"int8 q (streamed) M={M}")
    assert_bf16_close(vq.float().cpu().numpy()[:, :, 40].reshape(M, C), qkv[:, 2 * C:], f"int8 v (streamed) M={M}")


@pytest.mark.parametrize("M", [1, 8])
def test_int8_fused_ops_7b_shapes(hip, M):
    """llm.int8 (wfmt 2) through every fused entry point the model uses, at the 7B shapes (C 4096,
    32 heads of 128, H 11008, V 32000) and the two decode batch classes (M 1 and 8): rms_1 (its own
    launch) + llj_i8_stats + llj_norm_qkv_rope (RoPE, KV write), llj_norm_swiglu, llj_linear_resid
    (mlp.c_proj at K 11008 with its own statistics) and llj_norm_linear (lm_head), against the
    oracle's LLM.int8() restatement on the same rows. Two activation columns are outliers (>= 6
    after the norm) so the fp16 side product runs."""
    rng = np.random.default_rng(900 + M)
    C, nh, H, V, S = 4096, 32, 11008, 32000, 64
    hs = C // nh
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    x = rng.standard_normal((M, C)).astype(np.float32)
    x[:, [17, 3001]] *= 30.0
    x = bf16(x)
    g = bf16(rng.uniform(0.5, 1.5, C))
    xd, gd = T(x, torch.bfloat16), T(g, torch.bfloat16)
    xn = torch.empty_like(xd)
    call(hip, "llj_rmsnorm", xd.data_ptr(), gd.data_ptr(), 1e-5, xn.data_ptr(), M, C, st())
    torch.cuda.synchronize()
    xnh = xn.float().cpu().numpy()

    def wq(N, K):
        W = bf16(rng.standard_normal((N, K)) * 0.02)
        Wd = T(W, torch.bfloat16)
        cb = torch.empty(N, K, dtype=torch.int8, device=dev)
        scb = torch.empty(N, dtype=torch.float32, device=dev)
        call(hip, "llj_i8_quant_weight", Wd.data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st())
        cbt = torch.empty_like(cb)
        call(hip, "llj_i8_repack", cb.data_ptr(), cbt.data_ptr(), N, K, st())
        torch.cuda.synchronize()
        return O.int8_quantize_weight(W), cbt, scb

    ws = torch.empty(max(hip.llj_i8_ws_bytes(M, C), hip.llj_i8_ws_bytes(M, H)), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", xn.data_ptr(), C, M, C, 6.0, ws.data_ptr(), st())
    # QKV + RoPE + KV write
    (cbq, scbq), cbqd, scbqd = wq(3 * C, C)
    rope = O.build_rope_cache(128, hs)
    pos = np.array([37], np.int32)
    q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(M, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    rd, pd = T(rope), T(pos)
    call(hip, "llj_norm_qkv_rope", 2, xn.data_ptr(), None, 1e-5, cbqd.data_ptr(), scbqd.data_ptr(), q.data_ptr(),
         kc.data_ptr(), vc.data_ptr(), rd.data_ptr(), pd.data_ptr(), M, 1, C, nh, S, 0, M, ws.data_ptr(), None, None, 0, st())
    # SwiGLU
    (cb1, scb1), cb1d, scb1d = wq(H, C)
    (cb2, scb2), cb2d, scb2d = wq(H, C)
    h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_norm_swiglu", 2, xn.data_ptr(), None, 1e-5, cb1d.data_ptr(), scb1d.data_ptr(), cb2d.data_ptr(),
         scb2d.data_ptr(), h.data_ptr(), M, H, C, ws.data_ptr(), 0, None, None, 0, st())
    # lm_head
    (cbh, scbh), cbhd, scbhd = wq(V, C)
    lg = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_norm_linear", 2, xn.data_ptr(), None, 1e-5, cbhd.data_ptr(), scbhd.data_ptr(), lg.data_ptr(), V,
         M, V, C, ws.data_ptr(), 0, None, None, 0, st())
    torch.cuda.synchronize()
    # oracle on the same normalized rows
    qkv = bf16(O.int8_linear(xnh, cbq, scbq))
    qe = O.apply_rope(qkv[:, :C].reshape(M, 1, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(M, 1, nh, hs), rope[pos])[:, 0]
    assert_bf16_close(q.float().cpu().numpy(), qe, f"int8 q M={M}")
    assert_bf16_close(kc.float().cpu().numpy()[:, :, pos[0]], ke, f"int8 k cache M={M}")
    assert_bf16_close(vc.float().cpu().numpy()[:, :, pos[0]], qkv[:, 2 * C:].reshape(M, nh, hs), f"int8 v M={M}")
    hexp = bf16(bf16(O.silu(bf16(O.int8_linear(xnh, cb1, scb1)))) * bf16(O.int8_linear(xnh, cb2, scb2)))
    assert_bf16_close(h.float().cpu().numpy(), hexp, f"int8 swiglu M={M}", rel=3e-2)
    lref = O.int8_linear(xnh, cbh, scbh)
    assert_bf16_close(lg.float().cpu().numpy(), lref, f"int8 lm_head M={M}")
    # same int8 codes on both sides: only the output rounding (bf16) and fp32 order remain
    rel = np.linalg.norm(lg.float().cpu().numpy() - lref) / np.linalg.norm(lref)
    print(f"[int8] lm_head M={M} rel {rel:.3e}")
    assert rel < 3e-3, rel
    # mlp.c_proj + residual with the statistics of h
    (cbd_, scbd_), cbdd, scbdd = wq(C, H)
    hh = h.float().cpu().numpy()
    call(hip, "llj_i8_stats", h.data_ptr(), H, M, H, 6.0, ws.data_ptr(), st())
    xr = xd.clone()
    call(hip, "llj_linear_resid", 2, h.data_ptr(), H, cbdd.data_ptr(), scbdd.data_ptr(), xr.data_ptr(), C, M, C, H,
         ws.data_ptr(), 0, None, st())
    torch.cuda.synchronize()
    assert_bf16_close(xr.float().cpu().numpy(), x + bf16(O.int8_linear(hh, cbd_, scbd_)), f"int8 resid M={M}")


@pytest.mark.parametrize("temperature,top_k", [(0.8, 200), (1.0, 50), (0.5, 2), (1.3, 0), (1.0, 32000)])
def test_sample_inverse_cdf_vs_oracle(hip, temperature, top_k):
    """llj_sample with given uniforms against the oracle's restatement of generate.py:66-74 (the
    draw as an inverse CDF at the same u): identical indices, except where u * sum lands within
    fp32 summation noise (1e-4 of the sum) of a CDF step (the sums are associated differently;
    with all 32000 tokens kept the steps are ~3e-5 apart, so such draws are frequent there)."""
    rng = np.random.default_rng(int(temperature * 10) + top_k)
    M, V = 6, 32000
    L = bf16(rng.standard_normal((M, V)) * 3)
    L[1, 100:140] = L[1].max()  # a tie block at the maximum (all kept by torch.topk + where)
    Ld = T(L, torch.bfloat16)
    out = torch.empty(M, dtype=torch.int32, device=dev)
    mism = 0
    for rep in range(40):
        u = rng.random(M).astype(np.float32)
        u[0] = 0.0 if rep == 0 else u[0]
        ud = T(u)
        call(hip, "llj_sample", Ld.data_ptr(), V, M, V, temperature, top_k, ud.data_ptr(), 0, out.data_ptr(), None, 0,
             None, st())
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for m in range(M):
            want, p = O.sample_inverse_cdf(L[m], temperature, top_k, float(u[m]))
            assert p[got[m]] > 0, "picked a filtered index"
            if got[m] != want:
                cdf = np.cumsum(p, dtype=np.float64)
                gap = np.abs(cdf - u[m] * cdf[-1]).min()
                assert gap < 1e-4 * cdf[-1], (rep, m, got[m], want, gap)
                mism += 1
    if 0 < top_k <= 200:  # a few hundred CDF steps: near-boundary draws are rare
        assert mism <= 2, mism


def test_sample_device_rng_distribution(hip):
    """The in-graph path (u from the counter hash of seed, position and row): 8192 rows of the same
    logits draw from the top_k = 8 softmax with the oracle's probabilities (4-sigma bound per
    token), and a different position gives different draws."""
    rng = np.random.default_rng(77)
    V, M, k, temp = 32000, 8192, 8, 0.7
    row = bf16(rng.standard_normal(V) * 2)
    L = T(np.broadcast_to(row, (M, V)).copy(), torch.bfloat16)
    out = torch.empty(M, dtype=torch.int32, device=dev)
    pos = torch.tensor([41], dtype=torch.int32, device=dev)
    call(hip, "llj_sample", L.data_ptr(), V, M, V, temp, k, None, 1234, out.data_ptr(), None, 0, pos.data_ptr(), st())
    torch.cuda.synchronize()
    draws = out.cpu().numpy()
    _, p = O.sample_inverse_cdf(row, temp, k, 0.5)
    p = p / p.sum()
    assert set(np.unique(draws)) <= set(np.nonzero(p)[0])
    freq = np.bincount(draws, minlength=V) / M
    for i in np.nonzero(p)[0]:
        assert abs(freq[i] - p[i]) < 4 * np.sqrt(p[i] * (1 - p[i]) / M) + 1e-3, (i, freq[i], p[i])
    pos.fill_(42)
    out2 = torch.empty_like(out)
    call(hip, "llj_sample", L.data_ptr(), V, M, V, temp, k, None, 1234, out2.data_ptr(), None, 0, pos.data_ptr(), st())
    torch.cuda.synchronize()
    assert (out2.cpu().numpy() != draws).mean() > 0.3


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128, 4 | (2 << 8)])
@pytest.mark.parametrize("M,N,K", [(17, 256, 128), (100, 4096, 4096), (300, 11008, 4096), (256, 4096, 11008),
                                   (129, 384, 1024)])
def test_gemm_linear_and_resid(hip, wfmt, M, N, K):
    """Prefill GEMM (llj_gemm_linear / llj_gemm_resid, MFMA 128 x 128 tiles) against the oracle:
    int4 W4P with the row-sum offset removal and bf16 weights, ragged M (rows past M are never
    stored), 7B shapes."""
    rng = np.random.default_rng(M + N + K + wfmt)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    out = torch.full((M + 1, N), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
    call(hip, "llj_gemm_linear", wfmt, xd.data_ptr(), K, Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         out.data_ptr(), N, M, N, K, st())
    x0 = bf16(rng.standard_normal((M, N)).astype(np.float32))
    xr = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_resid", wfmt, xd.data_ptr(), K, Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         xr.data_ptr(), N, M, N, K, st())
    torch.cuda.synchronize()
    y = x @ Wref.T
    o = out.float().cpu().numpy()
    assert_bf16_close(o[:M], y, f"gemm wfmt={wfmt} M={M} N={N} K={K}")
    assert (o[M] == 7.0).all(), "wrote past row M"
    assert_bf16_close(xr.float().cpu().numpy(), x0 + bf16(y), f"gemm resid wfmt={wfmt}")


GLDS_TILES = {"256x256": {3: 1, 4: 1000}, "256x128": {3: 1, 4: 0}, "regstaged": {3: 0}}  # LLJ_OPT_GEMM_GLDS / _COST128


@pytest.fixture
def glds_tile(request, hip):
    """The prefill GEMM's M >= 256 kernel forced through its host-side options (llj_set_option): the
    LDS-DMA kernel's 256 x 256 or 256 x 128 tiles, or the register-staged kernel."""
    old = {k: hip.llj_set_option(k, v) for k, v in GLDS_TILES[request.param].items()}
    assert -1000 not in old.values()
    yield request.param
    for k, v in old.items():
        hip.llj_set_option(k, v)


@pytest.mark.parametrize("glds_tile", list(GLDS_TILES), indirect=True)
@pytest.mark.parametrize("wfmt", [0, 1])
@pytest.mark.parametrize("M,N,K", [(256, 512, 256), (300, 4096, 4096), (520, 11008, 4096), (257, 4096, 11008),
                                   (256, 256, 128), (384, 512, 384)])
def test_gemm_glds_tiles(hip, glds_tile, wfmt, M, N, K):
    """The LDS-DMA prefill GEMM (global_load_lds staging, counted vmcnt, source-swizzled LDS image,
    int4 row sums from the A fragments) in both tile shapes and the register-staged kernel, int4
    W4P and bf16 weights, against the oracle: store and residual epilogues, ragged M (a partial
    last row tile: rows past M clamped, never stored), K from 4 to 172 chunks."""
    rng = np.random.default_rng(M + N + K + wfmt)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    out = torch.full((M + 1, N), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
    call(hip, "llj_gemm_linear", wfmt, xd.data_ptr(), K, Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         out.data_ptr(), N, M, N, K, st())
    x0 = bf16(rng.standard_normal((M, N)).astype(np.float32))
    xr = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_resid", wfmt, xd.data_ptr(), K, Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         xr.data_ptr(), N, M, N, K, st())
    torch.cuda.synchronize()
    y = x @ Wref.T
    o = out.float().cpu().numpy()
    assert_bf16_close(o[:M], y, f"gemm {glds_tile} wfmt={wfmt} M={M} N={N} K={K}")
    assert (o[M] == 7.0).all(), "wrote past row M"
    assert_bf16_close(xr.float().cpu().numpy(), x0 + bf16(y), f"gemm resid {glds_tile} wfmt={wfmt}")


ZINT4 = _hip.WF_ZINT  # int4 with integral zeros: the convert-once LDS-DMA kernel at M >= 256


@pytest.mark.parametrize("M,N,K", [(256, 512, 256), (300, 4096, 4096), (520, 11008, 4096), (257, 4096, 11008),
                                   (2048, 12288, 4096), (100, 384, 1024), (256, 256, 128), (512, 384, 384)])
def test_gemm_w4z_convert_once(hip, M, N, K):
    """int4 prompt GEMM with LLJ_WF_ZINT (each chunk's codes converted once per workgroup into a bf16
    (q - z) tile, the scale in the epilogue; M < 256 takes the default int4 kernel) against the
    oracle, store and residual epilogues, ragged M; and the same call with the option off (the
    default int4 kernel) within bf16 rounding of it."""
    rng = np.random.default_rng(M + N + K + 5)
    Wref, Wd, szd = quant_operands(hip, rng, ZINT4, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    outs = []
    for w4z in (1, 0):
        old = hip.llj_set_option(_hip.OPT_GEMM_W4Z, w4z)
        out = torch.full((M + 1, N), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
        call(hip, "llj_gemm_linear", ZINT4, xd.data_ptr(), K, Wd.data_ptr(), szd.data_ptr(), out.data_ptr(), N, M, N,
             K, st())
        hip.llj_set_option(_hip.OPT_GEMM_W4Z, old)
        torch.cuda.synchronize()
        outs.append(out.float().cpu().numpy())
    y = x @ Wref.T
    o = outs[0]
    assert_bf16_close(o[:M], y, f"gemm w4z M={M} N={N} K={K}")
    assert (o[M] == 7.0).all(), "wrote past row M"
    assert_bf16_close(outs[1][:M], o[:M], f"gemm w4z vs default int4 M={M}")
    x0 = bf16(rng.standard_normal((M, N)).astype(np.float32))
    xr = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_resid", ZINT4, xd.data_ptr(), K, Wd.data_ptr(), szd.data_ptr(), xr.data_ptr(), N, M, N, K,
         st())
    torch.cuda.synchronize()
    assert_bf16_close(xr.float().cpu().numpy(), x0 + bf16(y), f"gemm w4z resid M={M}")


def test_gemm_w4z_exact_on_integer_rows(hip):
    """The convert-once tile is exact: with small-integer activations every product and fp32 partial
    sum is an integer below 2^24, so the GEMM is bitwise bf16(s * sum_k a (q - z))."""
    rng = np.random.default_rng(606)
    M, N, K = 512, 1024, 4096
    qw, sc, z = rand_w4(rng, N, K)
    Wd, szd = repack(hip, qw), sz_of(hip, sc, z)
    a = rng.integers(-4, 5, size=(M, K)).astype(np.float32)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_linear", ZINT4, T(a, torch.bfloat16).data_ptr(), K, Wd.data_ptr(), szd.data_ptr(),
         out.data_ptr(), N, M, N, K, st())
    torch.cuda.synchronize()
    codes = np.empty((N, K), dtype=np.int64)
    codes[:, 0::2] = qw & 15
    codes[:, 1::2] = qw >> 4
    acc = a.astype(np.int64) @ (codes - z.astype(np.int64)).T  # exact integers
    want = bf16(sc.reshape(1, N).astype(np.float32) * acc.astype(np.float32))
    np.testing.assert_array_equal(out.float().cpu().numpy(), want)


@pytest.mark.parametrize("M,H,K", [(256, 2816, 1024), (300, 11008, 4096), (2048, 11008, 4096), (520, 4096, 11008),
                                   (256, 128, 128)])
def test_gemm_swiglu_dual_pass(hip, M, H, K):
    """llj_gemm_swiglu (c_fc1 and c_fc2 of integral-zero int4 weights in one pass, one A tile for both,
    silu * mul in the epilogue) against the oracle, and bitwise equal to the two-pass form
    (llj_gemm_linear + llj_gemm_silu_mul with LLJ_WF_ZINT: the same per-element accumulation)."""
    rng = np.random.default_rng(M + H + K)
    W1, W1d, s1 = quant_operands(hip, rng, ZINT4, H, K)
    W2, W2d, s2 = quant_operands(hip, rng, ZINT4, H, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    h1 = torch.full((M + 1, H), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
    call(hip, "llj_gemm_swiglu", ZINT4, xd.data_ptr(), K, W1d.data_ptr(), s1.data_ptr(), W2d.data_ptr(), s2.data_ptr(),
         h1.data_ptr(), H, M, H, K, st())
    h2 = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_linear", ZINT4, xd.data_ptr(), K, W1d.data_ptr(), s1.data_ptr(), h2.data_ptr(), H, M, H, K, st())
    call(hip, "llj_gemm_silu_mul", ZINT4, xd.data_ptr(), K, W2d.data_ptr(), s2.data_ptr(), h2.data_ptr(), H, M, H, K,
         st())
    torch.cuda.synchronize()
    got = h1.float().cpu().numpy()
    assert (got[M] == 7.0).all(), "wrote past row M"
    np.testing.assert_array_equal(got[:M], h2.float().cpu().numpy())
    hexp = bf16(bf16(O.silu(bf16(x @ W1.T))) * bf16(x @ W2.T))
    assert_bf16_close(got[:M], hexp, f"gemm swiglu dual M={M}", rel=3e-2)


@pytest.mark.parametrize("M,H,K,tail", [(2048, 11008, 4096, 12), (512, 11008, 4096, 44), (300, 11008, 1024, 44),
                                        (768, 5632, 2048, 3), (1024, 11008, 4096, 0), (256, 2816, 1024, 0)])
def test_gemm_swiglu_tail_split(hip, M, H, K, tail):
    """llj_gemm_swiglu_ws: the dual pass's partial last wave of column tiles (the right `tail` x 64 columns of
    h at 256 CUs) as two K halves + a reduce, the rest on whole waves. Against the oracle; the whole-wave
    columns bitwise equal to llj_gemm_swiglu, the tail's within bf16 rounding of it (two fp32 partials);
    no split (0 bytes) where the tail would not fit one wave or there is none."""
    L = hip
    nb = L.llj_gemm_swiglu_ws_bytes(ZINT4, M, H, K)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if cus == 256:
        assert nb == 16 * M * 64 * tail
    assert L.llj_gemm_swiglu_ws_bytes(0, M, H, K) == 0  # int4 without integral zeros: no dual pass
    rng = np.random.default_rng(M + H + K + 1)
    W1, W1d, s1 = quant_operands(hip, rng, ZINT4, H, K)
    W2, W2d, s2 = quant_operands(hip, rng, ZINT4, H, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    ws = torch.full((max(nb, 4) // 4,), float("nan"), dtype=torch.float32, device=dev)
    h1 = torch.full((M + 1, H), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
    call(hip, "llj_gemm_swiglu_ws", ZINT4, xd.data_ptr(), K, W1d.data_ptr(), s1.data_ptr(), W2d.data_ptr(),
         s2.data_ptr(), h1.data_ptr(), H, M, H, K, ws.data_ptr(), nb, st())
    h2 = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_swiglu", ZINT4, xd.data_ptr(), K, W1d.data_ptr(), s1.data_ptr(), W2d.data_ptr(), s2.data_ptr(),
         h2.data_ptr(), H, M, H, K, st())
    torch.cuda.synchronize()
    got, one = h1.float().cpu().numpy(), h2.float().cpu().numpy()
    assert (got[M] == 7.0).all(), "wrote past row M"
    got = got[:M]
    Hc = H - 64 * (nb // (16 * M * 64) if nb else 0)
    np.testing.assert_array_equal(got[:, :Hc], one[:, :Hc])
    if Hc < H:
        assert_bf16_close(got[:, Hc:], one[:, Hc:], f"swiglu tail vs one pass M={M}", rel=3e-2)
    hexp = bf16(bf16(O.silu(bf16(x @ W1.T))) * bf16(x @ W2.T))
    assert_bf16_close(got, hexp, f"gemm swiglu tail split M={M}", rel=3e-2)


@pytest.mark.parametrize("wfmt", [1, ZINT4])
@pytest.mark.parametrize("M,N,K", [(256, 4096, 4096), (512, 4096, 11008), (300, 1024, 1024), (1024, 4096, 2048)])
def test_gemm_resid_split_k(hip, wfmt, M, N, K):
    """llj_gemm_resid_ws (K split over workgroups for few row tiles, fp32 partials reduced in slice order
    with the residual) against the oracle and against the unsplit llj_gemm_resid (same inputs, within
    bf16 rounding: the fp32 sums differ in order only); a workspace short by 4 bytes is refused."""
    L = hip
    nb = L.llj_gemm_resid_ws_bytes(wfmt, M, N, K)
    assert nb > 0, "this shape is expected to split"
    rng = np.random.default_rng(M + N + K + wfmt)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, N, K)
    x = bf16(rng.standard_normal((M, K)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    x0 = bf16(rng.standard_normal((M, N)).astype(np.float32))
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    ws = torch.empty(nb // 4, dtype=torch.float32, device=dev)
    assert L.llj_gemm_resid_ws(wfmt, xd.data_ptr(), K, Wd.data_ptr(), P(szd), T(x0, torch.bfloat16).data_ptr(), N, M, N,
                               K, ws.data_ptr(), nb - 4, st()) == 1000
    xr = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_resid_ws", wfmt, xd.data_ptr(), K, Wd.data_ptr(), P(szd), xr.data_ptr(), N, M, N, K, ws.data_ptr(),
         nb, st())
    xu = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_resid", wfmt, xd.data_ptr(), K, Wd.data_ptr(), P(szd), xu.data_ptr(), N, M, N, K, st())
    torch.cuda.synchronize()
    got = xr.float().cpu().numpy()
    assert_bf16_close(got, x0 + bf16(x @ Wref.T), f"gemm resid split-K wfmt={wfmt} M={M}")
    assert_bf16_close(got, xu.float().cpu().numpy(), f"gemm resid split-K vs unsplit wfmt={wfmt} M={M}")


def test_gemm_resid_split_k_plan(hip):
    """The split plan: none at 7B's 2048-row windows (256 tiles fill the CUs) or below 256 rows."""
    L = hip
    assert L.llj_gemm_resid_ws_bytes(ZINT4, 2048, 4096, 11008) == 0
    assert L.llj_gemm_resid_ws_bytes(1, 128, 4096, 4096) == 0
    assert L.llj_gemm_resid_ws_bytes(0, 512, 4096, 4096) == 0  # int4 without integral zeros: no LDS-DMA form
    assert L.llj_gemm_resid_ws_bytes(ZINT4, 512, 4096, 4096) > 0


def test_gemm_swiglu_dual_refuses(hip):
    """The one-pass form takes only integral-zero int4 at M >= 256 and H % 64 == 0 (EINVAL otherwise)."""
    L = hip
    z = torch.zeros(16, dtype=torch.uint8, device=dev)
    for wf, M, H in ((0, 256, 128), (ZINT4, 255, 128), (ZINT4, 256, 96), (1 | ZINT4, 256, 128)):
        assert L.llj_gemm_swiglu(wf, z.data_ptr(), 128, z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr(),
                                 z.data_ptr(), H, M, H, 128, st()) == 1000


@pytest.mark.parametrize("glds_tile", ["256x256", "256x128"], indirect=True)
@pytest.mark.parametrize("wfmt", [0, 1, ZINT4])
def test_gemm_glds_qkv_swiglu(hip, glds_tile, wfmt):
    """The LDS-DMA GEMM's QKV + RoPE + KV-write and silu * mul epilogues in both tile shapes
    (M = 2 x 150 prompt rows, 8 heads of 128; SwiGLU hidden 2816 = 11 x 256)."""
    rng = np.random.default_rng(90 + wfmt)
    B, T_, nh, hs, S = 2, 150, 8, 128, 256
    C, M = nh * hs, B * T_
    x = bf16(rng.standard_normal((M, C)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    rope = O.build_rope_cache(512, hs)
    pos = np.arange(5, 5 + T_, dtype=np.int32)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, 3 * C, C)
    q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(B, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    rd, pd = T(rope), T(pos)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    call(hip, "llj_gemm_qkv_rope", wfmt, xd.data_ptr(), Wd.data_ptr(), P(szd), q.data_ptr(), kc.data_ptr(),
         vc.data_ptr(), rd.data_ptr(), pd.data_ptr(), B, T_, C, nh, S, st())
    H = 2816
    W1, W1d, s1 = quant_operands(hip, rng, wfmt, H, C)
    W2, W2d, s2 = quant_operands(hip, rng, wfmt, H, C)
    h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_linear", wfmt, xd.data_ptr(), C, W1d.data_ptr(), P(s1), h.data_ptr(), H, M, H, C, st())
    call(hip, "llj_gemm_silu_mul", wfmt, xd.data_ptr(), C, W2d.data_ptr(), P(s2), h.data_ptr(), H, M, H, C, st())
    torch.cuda.synchronize()
    qkv = bf16(x @ Wref.T)
    qe = O.apply_rope(qkv[:, :C].reshape(B, T_, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(B, T_, nh, hs), rope[pos])
    ve = qkv[:, 2 * C:].reshape(B, T_, nh, hs)
    assert_bf16_close(q.float().cpu().numpy(), qe, f"gemm q {glds_tile}")
    kcn, vcn = kc.float().cpu().numpy(), vc.float().cpu().numpy()
    slots = pos % S
    assert_bf16_close(kcn[:, :, slots].transpose(0, 2, 1, 3), ke, f"gemm k cache {glds_tile}")
    assert_bf16_close(vcn[:, :, slots].transpose(0, 2, 1, 3), ve, f"gemm v cache {glds_tile}")
    hexp = bf16(bf16(O.silu(bf16(x @ W1.T))) * bf16(x @ W2.T))
    assert_bf16_close(h.float().cpu().numpy(), hexp, f"gemm swiglu {glds_tile}", rel=3e-2)


@pytest.mark.parametrize("wfmt", [1, ZINT4])
@pytest.mark.parametrize("B,T_,nh,hs,S,p0", [(2, 150, 4, 64, 256, 200), (1, 257, 8, 128, 512, 0), (3, 100, 2, 128, 128, 60)])
def test_gemm_glds_qkv_lds_epilogue(hip, wfmt, B, T_, nh, hs, S, p0):
    """The 256 x 128 LDS-DMA GEMM's QKV epilogue through LDS (8 columns = 4 RoPE pairs per thread, one
    16-byte store): head sizes 64 / 128, ring slots wrapping past S, ragged last tile, several sequences;
    cache slots the prompt does not cover stay untouched."""
    rng = np.random.default_rng(7 * T_ + hs + p0 + (wfmt & 1))
    C, M = nh * hs, B * T_
    x = bf16(rng.standard_normal((M, C)).astype(np.float32))
    rope = O.build_rope_cache(p0 + T_ + 8, hs)
    pos = np.arange(p0, p0 + T_, dtype=np.int32)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, 3 * C, C)
    q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(B, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    xd, rd, pd = T(x, torch.bfloat16), T(rope), T(pos)
    call(hip, "llj_gemm_qkv_rope", wfmt, xd.data_ptr(), Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rd.data_ptr(), pd.data_ptr(), B, T_, C, nh, S, st())
    torch.cuda.synchronize()
    qkv = bf16(x @ Wref.T)
    qe = O.apply_rope(qkv[:, :C].reshape(B, T_, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(B, T_, nh, hs), rope[pos])
    ve = qkv[:, 2 * C:].reshape(B, T_, nh, hs)
    assert_bf16_close(q.float().cpu().numpy(), qe, "gemm q (LDS epilogue)")
    kcn, vcn = kc.float().cpu().numpy(), vc.float().cpu().numpy()
    slots = pos % S
    assert_bf16_close(kcn[:, :, slots].transpose(0, 2, 1, 3), ke, "gemm k cache (LDS epilogue)")
    assert_bf16_close(vcn[:, :, slots].transpose(0, 2, 1, 3), ve, "gemm v cache (LDS epilogue)")
    rest = np.setdiff1d(np.arange(S), slots)
    assert not kcn[:, :, rest].any() and not vcn[:, :, rest].any()


def _i8_operands(hip, W):
    """CB / SCB of an LLM.int8 weight (llj_i8_quant_weight, checked against the oracle's rule) and
    CB re-tiled into I8P (what Linear8bitLt holds on the device)."""
    N, K = W.shape
    cb = torch.empty(N, K, dtype=torch.int8, device=dev)
    scb = torch.empty(N, dtype=torch.float32, device=dev)
    call(hip, "llj_i8_quant_weight", T(W, torch.bfloat16).data_ptr(), 1, cb.data_ptr(), scb.data_ptr(), N, K, st())
    cbt = torch.empty_like(cb)
    call(hip, "llj_i8_repack", cb.data_ptr(), cbt.data_ptr(), N, K, st())
    torch.cuda.synchronize()
    cb_ref, scb_ref = O.int8_quantize_weight(W)
    np.testing.assert_array_equal(cb.cpu().numpy(), cb_ref)
    return cbt, scb, cb_ref, scb_ref


def _i8_act(rng, M, K, outliers):
    x = rng.standard_normal((M, K)).astype(np.float32)
    if outliers:
        x[:, rng.choice(K, outliers, replace=False)] *= 25.0
    return bf16(x)


@pytest.mark.parametrize("M,K", [(32, 4096), (300, 4096), (64, 11008), (2048, 4096)])
def test_i8_stats_many_rows(hip, M, K):
    """llj_i8_stats for prompt rows (M >= 32: the 2-D pass 1 with atomic column flags, then the row
    quantization with the list compaction): every byte of the workspace against the numpy
    restatement of the LLM.int8() rules."""
    rng = np.random.default_rng(M + K)
    x = _i8_act(rng, M, K, 7)
    x[M // 2, 5] = 40.0  # an outlier column set by one row only
    ws = torch.full((hip.llj_i8_ws_bytes(M, K),), 0xAB, dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", T(x, torch.bfloat16).data_ptr(), K, M, K, 6.0, ws.data_ptr(), st())
    torch.cuda.synchronize()
    _check_i8_ws(ws.cpu().numpy(), x, M, K)


def _i8_gather(hip, xd, M, K, ws, weights, on):
    """(ao16, [w16], kpad) pointers for llj_gemm_i8_* (the pre-gathered outlier matrices), or Nones.
    on: True = capacity for every column as the model sizes it (model.py _i8_gathered), "cap64" = a
    64-column capacity (more outliers than that: nothing gathered, the GEMM's per-tile side product)."""
    if not on:
        return None, [None] * len(weights), 0, []
    from lit_llama.model import I8_GATHER_MAX

    kpad = 64 if on == "cap64" else min((K + 63) // 64 * 64, I8_GATHER_MAX)
    ao = torch.full((M, kpad), float("nan"), dtype=torch.float16, device=dev)  # past the pad: never read
    call(hip, "llj_i8_gather_act", xd.data_ptr(), K, M, K, ws.data_ptr(), ao.data_ptr(), kpad, st())
    keep, ptrs = [ao], []
    for cbt, scb, N in weights:
        t = torch.full((N, kpad), float("nan"), dtype=torch.float16, device=dev)
        call(hip, "llj_i8_gather_weight", cbt.data_ptr(), scb.data_ptr(), N, K, ws.data_ptr(), t.data_ptr(), kpad, st())
        keep.append(t)
        ptrs.append(t.data_ptr())
    return ao.data_ptr(), ptrs, kpad, keep


@pytest.mark.parametrize("gather", [False, True, "cap64"])
@pytest.mark.parametrize("outliers", [0, 6, 300])
@pytest.mark.parametrize("M,N,K", [(40, 256, 4096), (300, 4096, 4096), (129, 384, 11008), (48, 256, 17920)])
def test_gemm_i8_linear_resid_silu(hip, M, N, K, outliers, gather):
    """LLM.int8() prefill GEMM (int8 MFMA over the quantized rows + the fp16 outlier side product;
    llj_gemm_i8_linear / _resid / _silu_mul) against the oracle's restatement (bitsandbytes absent:
    parity unpinned) and against the int8 GEMV on the same workspace; the side product either
    gathered per tile or as a dense f16 GEMM over the pre-gathered outlier matrices (gather), also
    past the gathers' capacity (cap64 with 300 columns) and at K = 17,920 (30B mlp.c_proj: the
    gathers' list capped at I8_GATHER_MAX entries of LDS)."""
    rng = np.random.default_rng(M + N + K + outliers)
    W = bf16(rng.standard_normal((N, K)) * 0.02)
    W2 = bf16(rng.standard_normal((N, K)) * 0.02)
    cbt, scb, cb_ref, scb_ref = _i8_operands(hip, W)
    cbt2, scb2, cb_ref2, scb_ref2 = _i8_operands(hip, W2)
    x = _i8_act(rng, M, K, outliers)
    xd = T(x, torch.bfloat16)
    ws = torch.empty(hip.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", xd.data_ptr(), K, M, K, 6.0, ws.data_ptr(), st())
    ao, (g1, g2), kp, keep = _i8_gather(hip, xd, M, K, ws, [(cbt, scb, N), (cbt2, scb2, N)], gather)
    out = torch.full((M + 1, N), 7.0, dtype=torch.bfloat16, device=dev)  # row M: canary
    call(hip, "llj_gemm_i8_linear", xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), ao, g1, kp,
         out.data_ptr(), N, M, N, K, st())
    x0 = bf16(rng.standard_normal((M, N)).astype(np.float32))
    xr = T(x0, torch.bfloat16)
    call(hip, "llj_gemm_i8_resid", xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), ao, g1, kp,
         xr.data_ptr(), N, M, N, K, st())
    gv = torch.empty(M, N, dtype=torch.bfloat16, device=dev)  # the int8 GEMV in 8-row slices (4 at K > 12k: LDS)
    sl = 8 if 8 * (K + 16) <= 96 * 1024 else 4
    for r0 in range(0, M, sl):
        r = min(sl, M - r0)
        call(hip, "llj_linear", 2, xd[r0].data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), None, gv[r0].data_ptr(), N, r,
             N, K, ws.data_ptr(), r0, None, st())
    h = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_i8_linear", xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), ao, g1, kp,
         h.data_ptr(), N, M, N, K, st())
    call(hip, "llj_gemm_i8_silu_mul", xd.data_ptr(), K, cbt2.data_ptr(), scb2.data_ptr(), ws.data_ptr(), ao, g2, kp,
         h.data_ptr(), N, M, N, K, st())
    torch.cuda.synchronize()
    ref = O.int8_linear(x, cb_ref, scb_ref)
    o = out.float().cpu().numpy()
    assert (o[M] == 7.0).all(), "wrote past row M"
    assert_bf16_close(o[:M], ref, f"gemm int8 M={M} N={N} K={K} outliers={outliers}", rel=2e-2)
    assert_bf16_close(o[:M], gv.float().cpu().numpy(), "gemm int8 vs GEMV", rel=2e-2)
    assert_bf16_close(xr.float().cpu().numpy(), x0 + bf16(ref), "gemm int8 resid", rel=2e-2)
    hexp = bf16(bf16(O.silu(bf16(ref))) * bf16(O.int8_linear(x, cb_ref2, scb_ref2)))
    assert_bf16_close(h.float().cpu().numpy(), hexp, "gemm int8 swiglu", rel=3e-2)


@pytest.mark.parametrize("gather", [False, True, "cap64"])
@pytest.mark.parametrize("B,T_,nh,hs,outliers", [(1, 200, 32, 128, 6), (3, 40, 4, 64, 0), (1, 300, 8, 128, 6)])
def test_gemm_i8_qkv_rope_kv(hip, B, T_, nh, hs, outliers, gather):
    """llj_gemm_i8_qkv_rope: LLM.int8 c_attn + RoPE + KV-cache write for a whole prompt."""
    rng = np.random.default_rng(B * T_ + 77)
    C, S = nh * hs, max(256, T_ + 8)  # no ring wrap: every slot written once
    M = B * T_
    x = _i8_act(rng, M, C, outliers)
    rope = O.build_rope_cache(512, hs)
    pos = np.arange(5, 5 + T_, dtype=np.int32)
    W = bf16(rng.standard_normal((3 * C, C)) * 0.02)
    cbt, scb, cb_ref, scb_ref = _i8_operands(hip, W)
    xd, rd, pd = T(x, torch.bfloat16), T(rope), T(pos)
    ws = torch.empty(hip.llj_i8_ws_bytes(M, C), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", xd.data_ptr(), C, M, C, 6.0, ws.data_ptr(), st())
    q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(B, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    ao, (g1,), kp, keep = _i8_gather(hip, xd, M, C, ws, [(cbt, scb, 3 * C)], gather)
    call(hip, "llj_gemm_i8_qkv_rope", xd.data_ptr(), cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), ao, g1, kp,
         q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rd.data_ptr(), pd.data_ptr(), B, T_, C, nh, S, st())
    torch.cuda.synchronize()
    qkv = bf16(O.int8_linear(x, cb_ref, scb_ref))
    qe = O.apply_rope(qkv[:, :C].reshape(B, T_, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(B, T_, nh, hs), rope[pos])
    ve = qkv[:, 2 * C:].reshape(B, T_, nh, hs)
    assert_bf16_close(q.float().cpu().numpy(), qe, "int8 gemm q", rel=2e-2)
    slots = pos % S
    kg = kc.float().cpu().numpy()[:, :, slots].transpose(0, 2, 1, 3)
    vg = vc.float().cpu().numpy()[:, :, slots].transpose(0, 2, 1, 3)
    assert_bf16_close(kg, ke, "int8 gemm k", rel=2e-2)
    assert_bf16_close(vg, ve, "int8 gemm v", rel=2e-2)


@pytest.mark.parametrize("M", [150, 300])
@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128, 4 | (2 << 8)])
def test_gemm_swiglu_two_pass(hip, wfmt, M):
    """c_fc1 into h (llj_gemm_linear), then c_fc2 with the silu * mul epilogue in place
    (llj_gemm_silu_mul): model.py:258 with the reference's bf16 rounding points. M = 300 takes
    the 256-row tiles (bf16 / int8, int4 where enabled)."""
    rng = np.random.default_rng(70 + wfmt + M)
    C, H = 1024, 2816
    W1, W1d, s1 = quant_operands(hip, rng, wfmt, H, C)
    W2, W2d, s2 = quant_operands(hip, rng, wfmt, H, C)
    x = bf16(rng.standard_normal((M, C)).astype(np.float32))
    xd = T(x, torch.bfloat16)
    h = torch.empty(M, H, dtype=torch.bfloat16, device=dev)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    call(hip, "llj_gemm_linear", wfmt, xd.data_ptr(), C, W1d.data_ptr(), P(s1), h.data_ptr(), H, M, H, C, st())
    call(hip, "llj_gemm_silu_mul", wfmt, xd.data_ptr(), C, W2d.data_ptr(), P(s2), h.data_ptr(), H, M, H, C, st())
    torch.cuda.synchronize()
    hexp = bf16(bf16(O.silu(bf16(x @ W1.T))) * bf16(x @ W2.T))
    assert_bf16_close(h.float().cpu().numpy(), hexp, f"gemm swiglu wfmt={wfmt}", rel=3e-2)


@pytest.mark.parametrize("wfmt", [0, 1, 3, W4G_128, 4 | (2 << 8)])
@pytest.mark.parametrize("B,T_,nh,hs", [(1, 200, 32, 128), (3, 40, 4, 64), (2, 150, 8, 128)])
def test_gemm_qkv_rope_kv(hip, wfmt, B, T_, nh, hs):
    """llj_gemm_qkv_rope: c_attn + RoPE + KV-cache write for a whole prompt (ring slots p % S)."""
    rng = np.random.default_rng(B * T_ + wfmt)
    C, S = nh * hs, 256
    M = B * T_
    x = bf16(rng.standard_normal((M, C)).astype(np.float32))
    rope = O.build_rope_cache(512, hs)
    pos = np.arange(5, 5 + T_, dtype=np.int32)
    Wref, Wd, szd = quant_operands(hip, rng, wfmt, 3 * C, C)
    q = torch.zeros(M, C, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(B, nh, S, hs, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    xd, rd, pd = T(x, torch.bfloat16), T(rope), T(pos)
    call(hip, "llj_gemm_qkv_rope", wfmt, xd.data_ptr(), Wd.data_ptr(), None if szd is None else szd.data_ptr(),
         q.data_ptr(), kc.data_ptr(), vc.data_ptr(), rd.data_ptr(), pd.data_ptr(), B, T_, C, nh, S, st())
    torch.cuda.synchronize()
    qkv = bf16(x @ Wref.T)
    qe = O.apply_rope(qkv[:, :C].reshape(B, T_, nh, hs), rope[pos]).reshape(M, C)
    ke = O.apply_rope(qkv[:, C:2 * C].reshape(B, T_, nh, hs), rope[pos])
    ve = qkv[:, 2 * C:].reshape(B, T_, nh, hs)
    assert_bf16_close(q.float().cpu().numpy(), qe, "gemm q")
    kcn, vcn = kc.float().cpu().numpy(), vc.float().cpu().numpy()
    slots = pos % S
    assert_bf16_close(kcn[:, :, slots].transpose(0, 2, 1, 3), ke, "gemm k cache")
    assert_bf16_close(vcn[:, :, slots].transpose(0, 2, 1, 3), ve, "gemm v cache")


@pytest.mark.parametrize("hs,nh,B,T_,S,p0", [(128, 4, 1, 200, 256, 0), (64, 4, 2, 130, 160, 17), (128, 2, 1, 64, 64, 0),
                                            (128, 3, 1, 33, 2048, 1000), (128, 2, 1, 700, 1024, 0)])
@pytest.mark.parametrize("pair", ["0", "1"])
@pytest.mark.parametrize("qb", ["1", "2"])
def test_attention_prefill_flash(hip, hs, nh, B, T_, S, p0, qb, pair):
    """The MFMA flash attention for prompt rows (llj_attention_prefill) against the oracle: causal
    over cache slots 0 .. p0 + t, partial last query block, ragged key tiles, earlier context (p0 > 0);
    one or two 16-query blocks per wave (LLJ_OPT_FLASH_QB) and one query block or a (long, short) pair
    per workgroup (LLJ_OPT_FLASH_PAIR; odd block counts leave the middle block alone)."""
    from lit_llama import _hip

    with option(hip, _hip.OPT_FLASH_QB, int(qb)), option(hip, _hip.OPT_FLASH_PAIR, int(pair)):
        _flash_case(hip, hs, nh, B, T_, S, p0)


def _flash_case(hip, hs, nh, B, T_, S, p0):
    rng = np.random.default_rng(hs + T_ + p0)
    C = nh * hs
    kc = bf16(rng.standard_normal((B, nh, S, hs)))
    vc = bf16(rng.standard_normal((B, nh, S, hs)))
    q = bf16(rng.standard_normal((B * T_, C)) * 2)
    pos = np.arange(p0, p0 + T_, dtype=np.int32)
    y = torch.empty(B * T_, C, dtype=torch.bfloat16, device=dev)
    qd, kd, vd, pd = T(q, torch.bfloat16), T(kc, torch.bfloat16), T(vc, torch.bfloat16), T(pos)
    call(hip, "llj_attention_prefill", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), y.data_ptr(), pd.data_ptr(), B, T_,
         nh, hs, S, st())
    torch.cuda.synchronize()
    # P is rounded to bf16 before the P.V MFMA (as flash kernels do): ~1 bf16 ulp on the weights
    assert_bf16_close(y.float().cpu().numpy(), _attn_oracle(q, kc, vc, pos, S, T_, nh, hs), "flash prefill", rel=2e-2)


@pytest.mark.parametrize("scale_kind", ["fp32", "bf16"])
def test_gemm_grouped_dequant_equals_get_weight_bf16(hip, scale_kind):
    """The grouped-int4 prefill GEMM dequantizes every B fragment to the reference's
    get_weight(bfloat16) value (quantization.py:390-409: (q - z) in bf16, times the scale in the
    scale's precision, stored to bf16) bit for bit, with fp32 scales (the fp32 GPTQ calibration's)
    as well as bf16 ones: an identity A makes the GEMM output the dequantized weight itself
    (one nonzero product per output, exact in the fp32 accumulator)."""
    rng = np.random.default_rng(11)
    N, K, g = 256, 384, 128
    qw, sc, z = rand_w4g(rng, N, K, g)
    if scale_kind == "bf16":
        sc = bf16(sc)
    x = np.eye(K, dtype=np.float32)
    out = torch.empty(K, N, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_gemm_linear", 4 | (1 << 8), T(x, torch.bfloat16).data_ptr(), K, repack(hip, qw).data_ptr(),
         sz_grouped(hip, sc, z).data_ptr(), out.data_ptr(), N, K, N, K, st())
    torch.cuda.synchronize()
    wref = O.colblock_get_weight(qw, sc, z, 4, tile_cols=g, bf16=True)
    np.testing.assert_array_equal(out.float().cpu().numpy().T, wref)


def _i8_ws_offsets(M, K):
    """Byte offsets of (cnt, list) in the statistics workspace (csrc/i8ws.h i8_offsets)."""
    a16 = lambda v: (v + 15) & ~15
    kb = ((K + 31) // 32 + 31) & ~31
    part = a16(16 + M * K)
    cnt = part + 4 * 32 * M
    return cnt, cnt + 4 * 32, kb


@pytest.mark.parametrize("M,K,outliers", [(8, 4096, 3), (8, 11008, 300), (64, 4096, 6)])
def test_int8_consumers_bound_stale_outlier_counts(hip, M, K, outliers):
    """Robustness (the r05i fault): a workspace whose per-k-block outlier counts exceed the list width
    kb and whose list holds columns outside [0, K) must not make the int8 consumers read out of bounds.
    The GEMV (decode rows: in-stream side product, the after-stream fast and general paths) and, for
    prompt rows, the gathers + the LLM.int8 GEMM take the counts clamped to kb and the columns clamped
    to [0, K): the call returns 0, the device reports no fault and the outputs are finite (their
    values are those of the clamped list, i.e. wrong by design, and are not checked)."""
    rng = np.random.default_rng(M + K + outliers)
    N = 256
    W = bf16(rng.standard_normal((N, K)) * 0.02)
    cbt, scb, _, _ = _i8_operands(hip, W)
    xd = T(_i8_act(rng, M, K, outliers), torch.bfloat16)
    ws = torch.empty(hip.llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
    call(hip, "llj_i8_stats", xd.data_ptr(), K, M, K, 6.0, ws.data_ptr(), st())
    torch.cuda.synchronize()
    cnt_off, list_off, kb = _i8_ws_offsets(M, K)
    ws[cnt_off:cnt_off + 4 * 32].view(torch.int32).fill_(1 << 20)  # every block "full" past kb
    lst = ws[list_off:list_off + 4 * 32 * kb].view(torch.int32)
    lst.copy_(torch.randint(-(1 << 30), 1 << 30, lst.shape, dtype=torch.int32, device=dev))
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    if M <= 8:
        call(hip, "llj_linear", 2, xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), None, out.data_ptr(), N, M, N, K,
             ws.data_ptr(), 0, None, st())
    else:
        ao, (g1,), kp, keep = _i8_gather(hip, xd, M, K, ws, [(cbt, scb, N)], True)
        call(hip, "llj_gemm_i8_linear", xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), ao, g1, kp,
             out.data_ptr(), N, M, N, K, st())
        out2 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
        call(hip, "llj_gemm_i8_linear", xd.data_ptr(), K, cbt.data_ptr(), scb.data_ptr(), ws.data_ptr(), None, None, 0,
             out2.data_ptr(), N, M, N, K, st())  # the per-tile side product (no gathers)
        torch.cuda.synchronize()
        assert torch.isfinite(out2.float()).all()
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()


@pytest.mark.parametrize("M,regime", [(1, "few"), (8, "few"), (8, "none")])
def test_int8_statistics_handoff_split_attention(hip, M, regime):
    """llj_attention_i8 over a long cache (nsplit > 1: key ranges per block, the statistics of y
    written by attention_combine_kernel, which also zeroes h's block): y equals llj_attention_split's
    output bitwise, y's SCA and outlier columns equal llj_i8_stats' bitwise, and h's block comes back
    zero. 7B head shape (32 heads x 128), S = 2048, p = 2000, 16 splits."""
    rng = np.random.default_rng(2100 + M + len(regime))
    C, nh, H, S, p0, nsplit = 4096, 32, 11008, 2048, 2000, 16
    hs = C // nh
    kc = T(bf16(rng.standard_normal((M, nh, S, hs))), torch.bfloat16)
    vv = rng.standard_normal((M, nh, S, hs)).astype(np.float32) * (0.5 if regime == "none" else 1.0)
    if regime == "few":
        vv[:, 5, :, 9] = 9.0  # one y column >= 6 in every row
    vc = T(bf16(vv), torch.bfloat16)
    q = T(bf16(rng.standard_normal((M, C))), torch.bfloat16)
    pos = T(np.array([p0], np.int32))
    ws = torch.empty(hip.llj_attention_ws_bytes(M, nh, hs, nsplit), dtype=torch.uint8, device=dev)
    y = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    y_st = torch.zeros(hip.llj_i8_rowstats_bytes(C) // 4, dtype=torch.int32, device=dev)
    h_st = torch.full((hip.llj_i8_rowstats_bytes(H) // 4,), 7, dtype=torch.int32, device=dev)  # to be zeroed
    call(hip, "llj_attention_i8", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), y.data_ptr(), pos.data_ptr(), M, 1, nh,
         hs, S, nsplit, ws.data_ptr(), y_st.data_ptr(), h_st.data_ptr(), h_st.numel(), 6.0, st())
    torch.cuda.synchronize()
    assert not h_st.any()
    y_ref = torch.empty_like(y)
    call(hip, "llj_attention_split", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), y_ref.data_ptr(), pos.data_ptr(), M, 1,
         nh, hs, S, nsplit, ws.data_ptr(), st())
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    sca_w, fl_w = _i8_ws_stats(hip, y, M, C)
    sca_s, fl_s = _st_decode(y_st, M, C)
    np.testing.assert_array_equal(sca_s, sca_w)
    np.testing.assert_array_equal(fl_s, fl_w)
    assert fl_s.any() == (regime == "few")


@pytest.mark.parametrize("nsplit,p0,S", [(2, 80, 144), (4, 80, 144), (4, 143, 144), (3, 300, 256), (4, 5, 144)])
def test_attention_part_merged_in_cproj(hip, nsplit, p0, S):
    """Decode attention of one row as nsplit interleaved key splits (llj_attention_part: block s takes
    the key groups s * 32 + 32 nsplit i) whose partials attn.c_proj merges in its prologue
    (llj_linear_resid_attn, wfmt 0 int4): x0 + bf16(y) . W^T against the oracle's attention + Linear, and
    against the one-block attention + llj_linear_resid within the bf16 bound (the splits sum the keys
    in another fp32 order). p0 >= S: the rolled ring; p0 = 5: most splits empty."""
    rng = np.random.default_rng(nsplit * 1000 + p0 + S)
    nh, hs = 32, 128
    C = nh * hs
    kc = bf16(rng.standard_normal((1, nh, S, hs)))
    vc = bf16(rng.standard_normal((1, nh, S, hs)))
    q = bf16(rng.standard_normal((1, C)) * 2)
    pos = np.array([p0], np.int32)
    qd, kd, vd, pd = T(q, torch.bfloat16), T(kc, torch.bfloat16), T(vc, torch.bfloat16), T(pos)
    part = torch.full((hip.llj_attention_ws_bytes(1, nh, hs, nsplit),), 0xFF, dtype=torch.uint8, device=dev)
    call(hip, "llj_attention_part", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), pd.data_ptr(), 1, 1, nh, hs, S, nsplit,
         part.data_ptr(), st())
    Wref, Wd, szd = quant_operands(hip, rng, 0, C, C)
    x0 = bf16(rng.standard_normal((1, C)))
    xa = T(x0, torch.bfloat16)
    call(hip, "llj_linear_resid_attn", 0, part.data_ptr(), nsplit, nh, Wd.data_ptr(), szd.data_ptr(), xa.data_ptr(), C,
         C, C, None, st())
    y = torch.empty(1, C, dtype=torch.bfloat16, device=dev)
    call(hip, "llj_attention", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), y.data_ptr(), pd.data_ptr(), 1, 1, nh, hs, S,
         st())
    xb = T(x0, torch.bfloat16)
    call(hip, "llj_linear_resid", 0, y.data_ptr(), C, Wd.data_ptr(), szd.data_ptr(), xb.data_ptr(), C, 1, C, C, None, 0,
         None, st())
    torch.cuda.synchronize()
    yo = bf16(_attn_oracle(q, kc, vc, pos, S, 1, nh, hs))
    # the partials themselves: the combine formula on the host gives the attention output
    pr = part.cpu().numpy().view(np.float32).reshape(nh, nsplit, hs + 4)
    Mx = pr[:, :, hs].max(1, keepdims=True)
    f = np.where(pr[:, :, hs] == -np.inf, 0.0, np.exp2(pr[:, :, hs] - Mx))
    ym = (pr[:, :, :hs] * f[..., None]).sum(1) / (pr[:, :, hs + 1] * f).sum(1, keepdims=True)
    assert_bf16_close(ym.reshape(1, C), yo, f"merged partials nsplit={nsplit} p={p0}", rel=2e-2)
    ref = x0 + bf16(yo.astype(np.float64) @ Wref.T.astype(np.float64))
    assert_bf16_close(xb.float().cpu().numpy(), ref, "one-block attention + resid", rel=2e-2)
    assert_bf16_close(xa.float().cpu().numpy(), ref, f"merged attn.c_proj nsplit={nsplit} p={p0}", rel=2e-2)
    assert_bf16_close(xa.float().cpu().numpy(), xb.float().cpu().numpy(), "merged vs one-block + resid", rel=2e-2)
