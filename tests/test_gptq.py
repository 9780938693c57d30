"""GPTQ producer (reference lit_llama/quantization.py:424-614).

CPU: the oracle restatement (oracle/gptq_np.py) against the reference's own GPTQQuantizer run
(tests/golden/gptq.npz, made by tests/golden/make_golden.py gen_gptq): Hessian, scales, zeros
and every packed byte identical. GPU: the column-loop kernel bitwise against the oracle's block
loop on the same running weights and Hinv; the pack kernel bitwise; the whole device
GPTQQuantizer against the reference's bytes, where the device Hessian GEMM and rocSOLVER
Cholesky may flip a rare code by one (bounded below)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import gptq_np as G

GOLD = np.load(Path(__file__).parent / "golden" / "gptq.npz")
CASES = ["a", "b", "c"]


def case(t):
    return (GOLD[f"{t}_W"], GOLD[f"{t}_X"], GOLD[f"{t}_H"], int(GOLD[f"{t}_bits"]), GOLD[f"{t}_quant_weight"],
            GOLD[f"{t}_scales"], GOLD[f"{t}_zeros"], float(GOLD[f"{t}_error"]))


def codes_of(qw: np.ndarray, bits: int) -> np.ndarray:
    epb = 8 // bits
    out = np.zeros((qw.shape[0], qw.shape[1] * epb), np.int32)
    for nr in range(epb):
        out[:, nr::epb] = (qw >> (nr * bits)) & ((1 << bits) - 1)
    return out


@pytest.mark.parametrize("t", CASES)
def test_oracle_matches_reference_gptq(t):
    W, X, H, bits, qw, sc, zr, err = case(t)
    Hh, n = np.zeros((W.shape[1],) * 2, np.float32), 0
    for j in range(X.shape[0]):  # one sample per hook call, as quantize/gptq.py:96-104
        Hh, n = G.collect_input_stats(Hh, n, X[j:j + 1])
    np.testing.assert_array_equal(Hh, H)
    Q, s, z, e = G.gptq_quantize(W, H, bits)
    np.testing.assert_array_equal(s, sc)
    np.testing.assert_array_equal(z, zr)
    np.testing.assert_array_equal(G.pack_weight(Q, s, z, bits), qw)
    assert e == pytest.approx(err, rel=1e-4)


OPTS = np.load(Path(__file__).parent / "golden" / "gptq_opts.npz")
OPT_CASES = ["sym", "pt", "b64", "b32", "b16"]


def opt_case(t):
    bs, perch, sym, act = (int(v) for v in OPTS[f"{t}_opts"])
    return (OPTS[f"{t}_W"], OPTS[f"{t}_X"], OPTS[f"{t}_H"], int(OPTS[f"{t}_bits"]), OPTS[f"{t}_quant_weight"],
            OPTS[f"{t}_scales"], OPTS[f"{t}_zeros"], float(OPTS[f"{t}_error"]), bs, bool(perch), bool(sym), bool(act))


@pytest.mark.parametrize("t", OPT_CASES)
def test_oracle_matches_reference_gptq_options(t):
    """sym=True, perchannel=False and blocksizes 64 / 32 / 16 (reference 475-514, 557): the oracle's
    Hessian, scales, zeros and packed bytes against the reference's own GPTQQuantizer run
    (tests/golden/gptq_opts.npz, make_golden.py gen_gptq_opts)."""
    W, X, H, bits, qw, sc, zr, err, bs, perch, sym, act = opt_case(t)
    Hh, n = np.zeros((W.shape[1],) * 2, np.float32), 0
    for j in range(X.shape[0]):
        Hh, n = G.collect_input_stats(Hh, n, X[j:j + 1])
    np.testing.assert_array_equal(Hh, H)
    Q, s, z, e = G.gptq_quantize(W, H, bits, blocksize=bs, actorder=act, perchannel=perch, sym=sym)
    np.testing.assert_array_equal(s, sc)
    np.testing.assert_array_equal(z, zr)
    np.testing.assert_array_equal(G.pack_weight(Q, s, z, bits), qw)
    assert e == pytest.approx(err, rel=1e-4)
    if sym:
        assert (zr == 2 ** (bits - 1)).all()
    if not perch:
        assert len(np.unique(sc)) == 1


def test_fixture_has_dead_column_and_actorder_case():
    W, X, H, *_ = case("a")
    assert np.diag(H)[5] == 0  # quantization.py:544-546 path
    assert len(np.unique(np.diag(case("b")[2]))) == case("b")[2].shape[0]  # no ties for the argsort


# ------------------------------------------------------------------------------- GPU
dev = "cuda"


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.gpu
@pytest.mark.parametrize("t", CASES)
def test_gptq_block_kernel_bitwise(hip, t):
    """llj_gptq_block on the oracle's running weights / Hinv of every block == the oracle's
    gptq_block (reconstructions, errors, losses), bit for bit."""
    W, X, H, bits, *_ = case(t)
    from lit_llama import _hip
    scale, zero = G.find_params_weight(W, bits)
    Hinv, perm, dead = G.hinv_upper(H)
    Wr = W.astype(np.float32).copy()
    Wr[:, dead] = 0
    Wr = Wr[:, perm]
    N, K = Wr.shape
    hd = torch.from_numpy(Hinv).to(dev)
    sd, zd = torch.from_numpy(scale).to(dev), torch.from_numpy(zero).to(dev)
    for i1 in range(0, K, 128):
        i2 = i1 + 128
        Q1, E1, L1 = G.gptq_block(Wr[:, i1:i2], Hinv[i1:i2, i1:i2], scale, zero, bits)
        wt = torch.from_numpy(np.ascontiguousarray(Wr.T)).to(dev)
        qt = torch.full((K, N), np.nan, dtype=torch.float32, device=dev)
        err = torch.empty(128, N, dtype=torch.float32, device=dev)
        loss = torch.zeros(N, dtype=torch.float32, device=dev)
        _hip.call("llj_gptq_block", hd.data_ptr(), K, i1, wt.data_ptr(), N, sd.data_ptr(), zd.data_ptr(), bits,
                  qt.data_ptr(), err.data_ptr(), loss.data_ptr(), _st())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(qt[i1:i2].cpu().numpy().T, Q1)
        np.testing.assert_array_equal(err.cpu().numpy().T, E1)
        np.testing.assert_allclose(loss.cpu().numpy(), L1.sum(1), rtol=1e-5)
        Wr[:, i2:] = (Wr[:, i2:] - (E1 @ Hinv[i1:i2, i2:]).astype(np.float32)).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [8192, 8273])
def test_gptq_block_kernel_wide_bitwise(hip, N):
    """Both launch shapes of llj_gptq_block (32 rows x 8 lanes for N <= 8192, 64 rows x 4 lanes
    above; 8273 also leaves a ragged last workgroup): the fixture's rows tiled to N rows (rows are
    independent), first block, bit for bit against the oracle's gptq_block of the original rows."""
    W, X, H, bits, *_ = case(CASES[0])
    from lit_llama import _hip
    scale, zero = G.find_params_weight(W, bits)
    Hinv, perm, dead = G.hinv_upper(H)
    Wr = W.astype(np.float32).copy()
    Wr[:, dead] = 0
    Wr = Wr[:, perm]
    n0, K = Wr.shape
    Q1, E1, L1 = G.gptq_block(Wr[:, :128], Hinv[:128, :128], scale, zero, bits)
    rep = lambda a: np.resize(a, (N,) + a.shape[1:])  # noqa: E731  (row r = original row r % n0)
    wt = torch.from_numpy(np.ascontiguousarray(rep(Wr).T)).to(dev)
    qt = torch.full((K, N), np.nan, dtype=torch.float32, device=dev)
    err = torch.empty(128, N, dtype=torch.float32, device=dev)
    loss = torch.zeros(N, dtype=torch.float32, device=dev)
    sd = torch.from_numpy(rep(scale)).to(dev)
    zd = torch.from_numpy(rep(zero)).to(dev)
    _hip.call("llj_gptq_block", torch.from_numpy(Hinv).to(dev).data_ptr(), K, 0, wt.data_ptr(), N, sd.data_ptr(),
              zd.data_ptr(), bits, qt.data_ptr(), err.data_ptr(), loss.data_ptr(), _st())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(qt[:128].cpu().numpy().T, rep(Q1))
    np.testing.assert_array_equal(err.cpu().numpy().T, rep(E1))
    np.testing.assert_allclose(loss.cpu().numpy(), rep(L1.sum(1)), rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [4, 8])
def test_colblock_pack_kernel_bitwise(hip, bits):
    from lit_llama import _hip
    rng = np.random.default_rng(bits)
    N, K = 80, 256
    scale = rng.uniform(0.01, 0.1, N).astype(np.float32)
    zero = rng.integers(0, 2 ** bits, N).astype(np.float32)
    q = rng.integers(-2, 2 ** bits + 2, (N, K)).astype(np.float32)  # includes clamped codes
    Q = (scale[:, None] * (q - zero[:, None])).astype(np.float32)
    qw = torch.zeros((K * bits // 8, N), dtype=torch.uint8, device=dev)
    qt = torch.from_numpy(np.ascontiguousarray(Q.T)).to(dev)
    sd, zd = torch.from_numpy(scale).to(dev), torch.from_numpy(zero).to(dev)  # alive until the sync
    _hip.call("llj_colblock_pack", qt.data_ptr(), K, N, sd.data_ptr(), zd.data_ptr(), bits, qw.data_ptr(), _st())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(qw.cpu().numpy().T, G.pack_weight(Q, scale, zero, bits))


@pytest.mark.gpu
@pytest.mark.parametrize("t", CASES)
def test_gptq_quantizer_matches_reference(hip, t):
    """The device GPTQQuantizer (hook over the calibration samples, quantize()) against the
    reference's own output: scales / zeros identical, every code within 1 of the reference's and
    at most 0.5 % of them different (device GEMM / rocSOLVER vs the reference's CPU LAPACK)."""
    from lit_llama.quantization import ColBlockQuantizedLinear, GPTQQuantizer
    W, X, H, bits, qw, sc, zr, err = case(t)
    N, K = W.shape
    lin = torch.nn.Linear(K, N, bias=False).to(dev)
    lin.weight.data = torch.from_numpy(W).to(dev)
    gq = GPTQQuantizer(lin, bits=bits, groupsize=-1, actorder=True)
    h = lin.register_forward_hook(gq.collect_input_stats)
    with torch.no_grad():
        for j in range(X.shape[0]):
            lin(torch.from_numpy(X[j:j + 1]).to(dev))
    h.remove()
    np.testing.assert_allclose(gq.H.cpu().numpy(), H, rtol=1e-5, atol=1e-5 * np.abs(H).max())
    qm, e = gq.quantize()
    assert isinstance(qm, ColBlockQuantizedLinear) and qm.quant_weight.stride() == (1, N)
    np.testing.assert_array_equal(qm.scales.cpu().numpy().reshape(-1), sc)
    np.testing.assert_array_equal(qm.zeros.cpu().numpy().reshape(-1), zr)
    got, ref = codes_of(qm.quant_weight.cpu().numpy(), bits), codes_of(qw, bits)
    assert np.abs(got - ref).max() <= 1
    assert (got != ref).mean() <= 5e-3
    assert e == pytest.approx(err, rel=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("t", OPT_CASES)
def test_gptq_quantizer_options_match_reference(hip, t):
    """GPTQQuantizer(sym=..., perchannel=..., blocksize=...) on the device against the reference's own
    run with those options (gptq_opts.npz): scales / zeros identical, every code within 1 of the
    reference's and at most 0.5 % different (device GEMM / rocSOLVER vs CPU LAPACK); and the column
    loop kernel at that block size bitwise against the oracle's on the oracle's running weights."""
    from lit_llama import _hip
    from lit_llama.quantization import GPTQQuantizer
    W, X, H, bits, qw, sc, zr, err, bs, perch, sym, act = opt_case(t)
    N, K = W.shape
    lin = torch.nn.Linear(K, N, bias=False).to(dev)
    lin.weight.data = torch.from_numpy(W).to(dev)
    gq = GPTQQuantizer(lin, bits=bits, perchannel=perch, sym=sym, blocksize=bs, groupsize=-1, actorder=act)
    h = lin.register_forward_hook(gq.collect_input_stats)
    with torch.no_grad():
        for j in range(X.shape[0]):
            lin(torch.from_numpy(X[j:j + 1]).to(dev))
    h.remove()
    qm, e = gq.quantize()
    np.testing.assert_array_equal(qm.scales.cpu().numpy().reshape(-1), sc)
    np.testing.assert_array_equal(qm.zeros.cpu().numpy().reshape(-1), zr)
    got, ref = codes_of(qm.quant_weight.cpu().numpy(), bits), codes_of(qw, bits)
    assert np.abs(got - ref).max() <= 1
    assert (got != ref).mean() <= 5e-3
    assert e == pytest.approx(err, rel=1e-2)
    # the kernel alone, block by block on the oracle's running weights
    scale, zero = G.find_params_weight(W, bits, perch, sym)
    Hinv, perm, dead = G.hinv_upper(H, act)
    Wr = W.astype(np.float32).copy()
    Wr[:, dead] = 0
    if perm is not None:
        Wr = Wr[:, perm]
    hd = torch.from_numpy(Hinv).to(dev)
    sd, zd = torch.from_numpy(scale).to(dev), torch.from_numpy(zero).to(dev)
    for i1 in range(0, K, bs):
        i2 = i1 + bs
        Q1, E1, L1 = G.gptq_block(Wr[:, i1:i2], Hinv[i1:i2, i1:i2], scale, zero, bits)
        wt = torch.from_numpy(np.ascontiguousarray(Wr.T)).to(dev)
        qt = torch.full((K, N), np.nan, dtype=torch.float32, device=dev)
        errb = torch.empty(bs, N, dtype=torch.float32, device=dev)
        loss = torch.zeros(N, dtype=torch.float32, device=dev)
        _hip.call("llj_gptq_block_bs", hd.data_ptr(), K, i1, bs, wt.data_ptr(), N, sd.data_ptr(), zd.data_ptr(), bits,
                  qt.data_ptr(), errb.data_ptr(), loss.data_ptr(), _st())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(qt[i1:i2].cpu().numpy().T, Q1)
        np.testing.assert_array_equal(errb.cpu().numpy().T, E1)
        Wr[:, i2:] = (Wr[:, i2:] - (E1 @ Hinv[i1:i2, i2:]).astype(np.float32)).astype(np.float32)


@pytest.mark.gpu
def test_blockwise_driver_quantizes_like_reference(hip):
    """llama_blockwise_quantization (quantize/gptq.py:36-148) on the int4_gptq fixture's model and
    calibration tokens (make_golden.py gen_int4_gptq), calibrating in fp32 as the reference run
    did: every Linear replaced by a ColBlockQuantizedLinear whose scales / zeros are the
    reference's and whose codes are the reference's within one step, on all but a few entries
    (device GEMM / Cholesky summation order, compounded over the blocks); the quantized model,
    loaded into a bf16 gptq.int4 model, gives the reference's quantized logits within bf16 noise."""
    from oracle import llama_np as O
    from oracle.weights import Cfg, make_params
    from lit_llama import LLaMA, LLaMAConfig
    from lit_llama.quantization import ColBlockQuantizedLinear
    from lit_llama.utils import EmptyInitOnDevice
    from quantize.gptq import llama_blockwise_quantization
    from tests.test_model_gpu import build

    g = np.load(Path(__file__).parent / "golden" / "int4_gptq.npz")
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=2048)
    seed = int(g["seed"])
    params = make_params(cfg, seed)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.float32):
        model = LLaMA(LLaMAConfig(block_size=128, vocab_size=2048, n_layer=2, n_head=4, n_embd=256))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    gen = torch.Generator().manual_seed(seed)
    calib = torch.randint(3, cfg.vocab_size, (4, cfg.block_size), generator=gen)  # as make_golden.py
    errs = llama_blockwise_quantization(model, calib, "cuda", bits=4)
    assert len(errs) == 5 * cfg.n_layer + 1 and np.all(np.isfinite(list(errs.values())))
    agree, within1 = {}, {}
    for k in [k[3:] for k in g.files if k.startswith("sd/") and k.endswith(".quant_weight")]:
        name = k[:-len(".quant_weight")]
        mod = model.get_submodule(name)
        assert isinstance(mod, ColBlockQuantizedLinear)
        sd = mod.state_dict()
        np.testing.assert_allclose(sd["scales"].cpu().numpy(), g["sd/" + name + ".scales"], rtol=1e-6)
        np.testing.assert_array_equal(sd["zeros"].cpu().numpy(), g["sd/" + name + ".zeros"])
        a, b = codes_of(sd["quant_weight"].cpu().numpy(), 4), codes_of(g["sd/" + k], 4)
        agree[k] = float((a == b).mean())
        within1[k] = float((np.abs(a.astype(int) - b) <= 1).mean())
    print("code agreement with the reference's GPTQ run:", agree)
    print("within one step:", within1)
    # block 0 sees the same inputs as the reference (the embedding): its codes are the reference's
    for k, v in agree.items():
        if k.startswith("transformer.h.0."):
            assert v > 0.999, (k, v)
    # later blocks calibrate on the outputs of quantized predecessors computed with another
    # summation order (device GEMMs / SDPA vs the reference's CPU run); GPTQ's error feedback
    # turns those last-bit differences into different rounding decisions further along a row
    # (measured on MI355X: 87-100 % equal, 96.5-100 % within one step)
    assert min(within1.values()) > 0.95, within1
    # the quantized checkpoint in a bf16 gptq.int4 model (the generate.py flow)
    qsd = {k: v for k, v in model.state_dict().items()}
    qm = build(cfg, params, mode="gptq.int4", packed={k: v.cpu().numpy() for k, v in qsd.items()
                                                      if k.endswith((".quant_weight", ".scales", ".zeros"))})
    idx = torch.from_numpy(g["prompt"][None].astype(np.int64)).cuda()
    ours = qm(idx).float().cpu().numpy()[0, -1]
    ref_q = g["fp32_logits_step0"]
    fp32 = O.OracleLLaMA(cfg, params).forward(g["prompt"][None].astype(np.int64))[0, -1]
    e_ours = np.linalg.norm(ours - fp32) / np.linalg.norm(fp32)
    e_ref = np.linalg.norm(ref_q - fp32) / np.linalg.norm(fp32)
    d_ref = np.linalg.norm(ours - ref_q) / np.linalg.norm(ref_q)
    print("relative logit error vs the fp32 model: ours", e_ours, "reference GPTQ", e_ref, "ours vs ref", d_ref)
    assert e_ours < 1.1 * e_ref + 1e-2, (e_ours, e_ref)  # as good a quantization as the reference's


@pytest.mark.gpu
def test_gptq_cli_writes_a_checkpoint_generate_loads(hip, tmp_path):
    """quantize/gptq.py main (reference quantize/gptq.py:150-237) end to end on a random 19M
    checkpoint: tokenizer + calibration text -> llama_blockwise_quantization -> torch.save; the
    written state dict loads strictly into an --quantize gptq.int4 model (the reference's
    generate.py flow) whose logits stay near the bf16 model's and whose greedy decode runs."""
    from tokenizers import Tokenizer as HFTok
    from tokenizers.models import WordLevel
    from tokenizers.pre_tokenizers import Whitespace
    from oracle.weights import Cfg, make_params
    from lit_llama import LLaMA
    from lit_llama.utils import EmptyInitOnDevice
    from quantize.gptq import main
    import generate as G

    cfg = Cfg(n_layer=6, n_head=8, n_embd=512, vocab_size=35000)  # llama_configs["19M"]
    params = make_params(cfg, 11)
    ck = tmp_path / "lit-llama.pth"
    torch.save({k: torch.from_numpy(v) for k, v in params.items()}, ck)
    words = [f"w{i}" for i in range(3, 3000)]
    tok = HFTok(WordLevel({"<pad>": 0, "<s>": 1, "</s>": 2, **{w: i + 3 for i, w in enumerate(words)}},
                          unk_token="<pad>"))
    tok.pre_tokenizer = Whitespace()
    tok.save(str(tmp_path / "tokenizer.json"))
    rng = np.random.default_rng(5)
    (tmp_path / "calib.txt").write_text(" ".join(rng.choice(words, 600)))
    errs = main(checkpoint_path=ck, tokenizer_path=tmp_path / "tokenizer.json", n_samples=2, dtype="float32",
                quantize="gptq.int4", calibration_path=tmp_path / "calib.txt", block_size=256)
    out = tmp_path / "llama-gptq.4bit.pth"
    assert out.is_file() and len(errs) == 5 * cfg.n_layer + 1

    sd = torch.load(out, map_location="cpu", weights_only=True)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.bfloat16, quantization_mode="gptq.int4"):
        qm = LLaMA.from_name("19M")
    qm.load_state_dict(sd)  # strict: every key the quantized model expects, nothing else
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.bfloat16):
        fm = LLaMA.from_name("19M")
    fm.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    idx = torch.from_numpy(rng.integers(3, 3000, (1, 16))).cuda()
    lq = qm.eval()(idx).float()[0, -1]
    lf = fm.eval()(idx).float()[0, -1]
    rel = float((lq - lf).norm() / lf.norm())
    print("relative logit error of the CLI-quantized 19M model:", rel)
    # sanity bound only: code parity is pinned by the tests above. Per-channel int4 on random
    # weights costs ~0.27 relative logit error over 2 layers (reference's own run, int4_gptq
    # fixture); over these 6 layers it compounds to ~0.55 (measured on MI355X).
    assert rel < 0.75, rel
    qm.reset_cache()
    y = G.generate(qm, idx[0], 8, top_k=1)
    assert y.shape[0] == 24


# ------------------------------------------------------------------ grouped scales (tile_cols = g)
GG = np.load(Path(__file__).parent / "golden" / "gptq_grouped.npz")
GCASES = ["g1", "g2"]


def gcase(t):
    return {k[len(t) + 1:]: GG[k] for k in GG.files if k.startswith(t + "_")}


@pytest.mark.parametrize("t", GCASES)
def test_oracle_grouped_colblock_matches_reference(t):
    """The reference's grouped ColBlockQuantizedLinear (tile_cols = g): per-group find_params_weight,
    pack_weight and get_weight reproduced exactly by the oracle. The fixture also records that the
    reference's own grouped GPTQ column loop raises (quantization.py:576), which is why the grouped
    producer below is checked against the oracle only (parity unpinned)."""
    c = gcase(t)
    W, g, sc, zr = c["W"], int(c["g"]), c["scales"], c["zeros"]
    K = W.shape[1]
    assert sc.shape == (W.shape[0], (K + g - 1) // g) and int(c["ref_quantize_raises"]) == 1
    col = np.arange(K) // g
    for j in range(sc.shape[1]):
        s, z = G.find_params_weight(W[:, j * g:(j + 1) * g], 4)
        np.testing.assert_array_equal(s, sc[:, j])
        np.testing.assert_array_equal(z, zr[:, j])
    q = np.clip(np.round(W / sc[:, col]).astype(np.float32) + zr[:, col], 0, 15)
    Wrec = (sc[:, col] * (q - zr[:, col])).astype(np.float32)
    np.testing.assert_array_equal(G.pack_weight(Wrec, sc, zr, 4, g), c["quant_weight"])
    from oracle import llama_np as O
    np.testing.assert_array_equal(O.colblock_get_weight(c["quant_weight"], sc, zr, 4, tile_cols=g), c["wdeq"])


@pytest.mark.parametrize("t", GCASES)
def test_oracle_grouped_gptq_properties(t):
    """Grouped GPTQ restatement: one group spanning all columns is the ungrouped algorithm exactly;
    group 0's params are find_params_weight of the untouched first columns; grouping lowers the loss."""
    c = gcase(t)
    W, X, g = c["W"], c["X"], int(c["g"])
    K = W.shape[1]
    H, n = np.zeros((K, K), np.float32), 0
    for j in range(X.shape[0]):
        H, n = G.collect_input_stats(H, n, X[j:j + 1])
    Qg, sg, zg, eg = G.gptq_quantize(W, H, 4, actorder=False, groupsize=g)
    QK, sK, zK, eK = G.gptq_quantize(W, H, 4, actorder=False, groupsize=K)
    Q1, s1, z1, e1 = G.gptq_quantize(W, H, 4, actorder=False)
    np.testing.assert_array_equal(QK, Q1)
    np.testing.assert_array_equal(sK[:, 0], s1)
    assert eK == e1
    s0, z0 = G.find_params_weight(W[:, :g], 4)
    np.testing.assert_array_equal(sg[:, 0], s0)
    assert eg < e1


@pytest.mark.gpu
@pytest.mark.parametrize("t", GCASES)
def test_grouped_colblock_module_vs_reference(hip, t):
    """Our ColBlockQuantizedLinear(tile_cols = g) loaded with the reference's grouped buffers:
    forward on the grouped int4 GEMV (wfmt 4) vs the reference's fp32 forward and the oracle's
    bf16-input product; get_weight and the state dict give the reference's buffers back after the
    in-place repack."""
    from lit_llama.quantization import ColBlockQuantizedLinear
    from tests.helpers import assert_bf16_close, bf16
    c = gcase(t)
    N, K, g = c["W"].shape[0], c["W"].shape[1], int(c["g"])
    m = ColBlockQuantizedLinear(K, N, False, bits=4, tile_cols=g).to(dev)
    m.load_state_dict({"quant_weight": torch.from_numpy(c["quant_weight"]), "scales": torch.from_numpy(c["scales"]),
                       "zeros": torch.from_numpy(c["zeros"])})
    assert m.wfmt == 4 | ((g // 128) << 8)
    for M in (1, 5):
        x = c[f"x{M}"]
        with torch.no_grad():
            y = m(torch.from_numpy(x).to(dev, torch.bfloat16)).float().cpu().numpy()
        assert_bf16_close(y, bf16(x).astype(np.float64) @ c["wdeq"].T.astype(np.float64), f"{t} M={M} vs oracle")
        ref = c[f"y{M}"]
        assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-2  # bf16 input rounding vs the fp32 reference
    sd = m.state_dict()
    np.testing.assert_array_equal(sd["quant_weight"].cpu().numpy(), c["quant_weight"])
    np.testing.assert_array_equal(m.get_weight(torch.float).cpu().numpy(), c["wdeq"])


@pytest.mark.gpu
@pytest.mark.parametrize("t", GCASES)
def test_grouped_gptq_quantizer_vs_oracle(hip, t):
    """Device GPTQQuantizer(groupsize = g, actorder off) against the oracle's grouped restatement
    (parity unpinned: the reference's grouped loop raises). Group 0's params are exact; later groups
    are found on weights the device GEMM / Cholesky updated, so at least 97 % of the (row, group)
    params agree, and where they do every code is within two steps and at most 1 % differ."""
    from lit_llama.quantization import GPTQQuantizer
    c = gcase(t)
    W, X, g = c["W"], c["X"], int(c["g"])
    N, K = W.shape
    lin = torch.nn.Linear(K, N, bias=False).to(dev)
    lin.weight.data = torch.from_numpy(W).to(dev)
    gq = GPTQQuantizer(lin, bits=4, groupsize=g, actorder=False)
    h = lin.register_forward_hook(gq.collect_input_stats)
    with torch.no_grad():
        for j in range(X.shape[0]):
            lin(torch.from_numpy(X[j:j + 1]).to(dev))
    h.remove()
    H = gq.H.cpu().numpy()
    qm, e = gq.quantize()
    Q, sg, zg, eo = G.gptq_quantize(W, H, 4, actorder=False, groupsize=g)
    assert qm.scales.shape == (N, (K + g - 1) // g) and qm.tile_cols == g
    got_s, got_z = qm.scales.cpu().numpy(), qm.zeros.cpu().numpy()
    np.testing.assert_array_equal(got_s[:, 0], sg[:, 0])
    np.testing.assert_array_equal(got_z[:, 0], zg[:, 0])
    # a code flipped by one in an earlier block (allowed below) feeds a different error into the
    # later columns, which can move a later group's min / max: such (row, group) params may differ
    same = (np.abs(got_s - sg) <= 1e-5 * np.abs(sg)) & (got_z == zg)
    assert same.mean() >= 0.97, same.mean()
    got = codes_of(qm.quant_weight.cpu().numpy(), 4)
    ref = codes_of(G.pack_weight(Q, sg, zg, 4, g), 4)
    keep = same[:, np.arange(K) // g]  # codes of the (row, group) pairs with the same params
    assert np.abs(got - ref)[keep].max() <= 2  # a flip's error feedback can move a later code of its row by 2
    assert (got != ref)[keep].mean() <= 1e-2
    assert e == pytest.approx(eo, rel=1e-2)
    x = torch.randn(3, K, device=dev, dtype=torch.bfloat16)
    with torch.no_grad():
        y = qm(x).float()
        yr = x.float() @ qm.get_weight(torch.float).t()
    assert (y - yr).norm() / yr.norm() < 1e-2
