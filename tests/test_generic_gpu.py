"""The any-shape path (csrc/generic.hip via LLaMA._blocks_generic / _head): configurations outside
the streaming kernels' tiling, which the reference runs and the fast path cannot --
  * the JA fork's own 125M (n_layer 12, n_head 10, n_embd 780: head 78, n_hidden 2304, vocab 35000;
    reference lit_llama/model.py:48-51);
  * the reference test's n_embd 32 / n_head 16 (head 2), 16 layers, block 64
    (reference tests/test_model.py:108-112, test_bfloat16_llama_init).
Logits against the oracle on the same weights, prefill rows and teacher-forced decode steps, bf16
weights and gptq.int4 (the ColBlockQuantizedLinear buffers used as stored, no repack).

Tolerance, as in tests/test_model_7b_gpu.py: twice the measured bf16 noise floor, i.e. the oracle
against ITSELF with its Linears / RMSNorm means summed in another valid order, on these very weights,
ids and steps (tools/noise_floor.py --generic, profiles/r03_noise_floor_generic.json). Deeper models
carry more of it than the 2-layer width tests: n_embd 32 x 16 layers floor max 2.87e-2 / mean
2.9e-3; 125M (12 layers) max 1.71e-2 (bf16) / 1.88e-2 (int4), mean <= 1.56e-2. Every row / step is
held to 2x the max and the mean over rows to 2x the floor mean."""
import numpy as np
import pytest
import torch

from oracle import llama_np as O
from oracle.weights import Cfg, make_params
from tests.test_model_7b_gpu import _check, _gpu_steps, _oracle_steps, oracle_linears

pytestmark = pytest.mark.gpu

REF_TEST = Cfg(block_size=64, vocab_size=32000, n_layer=16, n_head=16, n_embd=32)
C125 = Cfg(block_size=128, n_layer=12, n_head=10, n_embd=780, vocab_size=35000)
# (max per row, mean over rows): 2x profiles/r03_noise_floor_generic.json
TOL_REF_TEST = (5.8e-2, 5.8e-3)
TOL_125M = (3.8e-2, 3.2e-2)
# llm.int8 re-quantizes every Linear input per row, so the same flips move whole int8 steps: floor max
# 3.12e-2 / mean 2.16e-2 (profiles/r04_noise_floor_generic.json, with the GPU-formula variant)
TOL_125M_I8 = (6.3e-2, 4.4e-2)


def _check_mean(got, ref, tol, what):
    worst = _check(got, ref, tol[0], what)
    B, n = got.shape[:2]
    mean = float(np.mean([np.linalg.norm(got[b, s] - ref[b, s]) / np.linalg.norm(ref[b, s])
                          for b in range(B) for s in range(n)]))
    assert mean < tol[1], f"{what}: mean rel err {mean:.3e}"
    return worst


def _setup(cfg: Cfg, mode, seed):
    from lit_llama import LLaMA, LLaMAConfig
    from lit_llama.utils import EmptyInitOnDevice

    pb, sd, lin = oracle_linears(make_params(cfg, seed), mode)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.bfloat16, quantization_mode=mode):
        m = LLaMA(LLaMAConfig(block_size=cfg.block_size, vocab_size=cfg.vocab_size, n_layer=cfg.n_layer,
                              n_head=cfg.n_head, n_embd=cfg.n_embd))
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    assert m._generic(), "this config should take the any-shape path"
    return m.eval(), O.OracleLLaMA(cfg, pb, linears=lin, act_bf16=True)


def test_reference_test_config_no_cache_vs_oracle():
    """The reference test's model (n_embd 32, head 2, 16 layers) at its batch 3 x 64 tokens,
    no-cache forward (all rows); then the cache path gives the same logits."""
    m, orc = _setup(REF_TEST, None, 32)
    idx = np.random.default_rng(3).integers(0, REF_TEST.vocab_size, (3, 64))
    out = m(torch.from_numpy(idx).cuda()).float().cpu().numpy()
    ref = orc.forward(idx)
    _check_mean(out, ref, TOL_REF_TEST, "ref-test config no-cache")
    m.reset_cache()
    out2 = m(torch.from_numpy(idx).cuda(), 64, torch.arange(64).cuda()).float().cpu().numpy()
    np.testing.assert_allclose(out2, out, rtol=0, atol=1e-6)


@pytest.mark.parametrize("mode", [None, "gptq.int4", "llm.int8"])
def test_125m_prefill_and_decode_vs_oracle(mode):
    """125M: a 12-token prompt (every row) then 4 teacher-forced decode steps, batch 2. llm.int8:
    Linear8bitLt at K = 780 / 2304 on the any-shape LLM.int8 kernels (llj_g_i8_linear)."""
    m, orc = _setup(C125, mode, 125)
    ids = np.random.default_rng(12).integers(3, C125.vocab_size, (2, 12 + 5))
    got, got_rows = _gpu_steps(m, ids, t_prompt=12, steps=4, s=32, all_rows=True)
    ref, ref_rows = _oracle_steps(orc, ids, t_prompt=12, steps=4, s=32, all_rows=True)
    tol = TOL_125M_I8 if mode == "llm.int8" else TOL_125M
    _check_mean(got_rows, ref_rows, tol, f"125M {mode} prompt rows")
    _check_mean(got, ref, tol, f"125M {mode} steps")


def test_125m_generate_graph_matches_eager_and_wraps():
    """generate() on 125M (greedy, the captured decode graph on the any-shape kernels): the same ids
    as a decode session stepped eagerly, past a ring wrap (max_seq_length 16 < 8 + 20 tokens)."""
    from lit_llama.engine import DecodeSession

    m, _ = _setup(C125, "gptq.int4", 7)
    prompt = torch.from_numpy(np.random.default_rng(5).integers(3, C125.vocab_size, 8)).cuda()
    outs = []
    for graph in (True, False):
        s = DecodeSession(m, 1, 16, 28, use_graph=graph)
        s.prefill(prompt.view(1, -1))
        s.decode(19)
        outs.append(s.output()[0].cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])
    assert outs[0].shape == (28,) and ((outs[0] >= 0) & (outs[0] < C125.vocab_size + 64)).all()


def test_generic_linear_grouped_int8_codes_vs_numpy():
    """llj_g_linear on ColBlock bits=8 codes with groups (tile_cols 256 over K 780 -> 4 groups, the
    last partial) and the residual form, against numpy (q - z) * s in fp32."""
    from lit_llama import _hip

    rng = np.random.default_rng(1)
    M, K, N, g = 5, 780, 36, 256
    G = (K + g - 1) // g
    q = rng.integers(0, 256, (N, K)).astype(np.uint8)
    sc = (rng.random((N, G)) * 0.01 + 0.001).astype(np.float32)
    zr = rng.integers(100, 156, (N, G)).astype(np.float32)
    x = O.bf16_round(rng.standard_normal((M, K)).astype(np.float32))
    res = O.bf16_round(rng.standard_normal((M, N)).astype(np.float32))
    Wd = (q.astype(np.float32) - np.repeat(zr, g, 1)[:, :K]) * np.repeat(sc, g, 1)[:, :K]
    ref = O.bf16_round(res + O.bf16_round(x @ Wd.T))
    dev = torch.device("cuda")
    qw = torch.from_numpy(q.T.copy()).to(dev)  # column-major (N, K) bytes: byte (n, k) at k*N + n
    xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
    y = torch.from_numpy(res).to(dev).to(torch.bfloat16)
    sct, zrt = torch.from_numpy(sc).to(dev), torch.from_numpy(zr).to(dev)
    _hip.call("llj_g_linear", 0, xt.data_ptr(), K, M, K, qw.data_ptr(), sct.data_ptr(), zrt.data_ptr(), 8, g, N,
              y.data_ptr(), N, y.data_ptr(), N, 0, _hip.stream())
    got = y.float().cpu().numpy()
    err = np.abs(got - ref).max() / np.abs(ref).max()
    print(f"[generic] grouped int8 linear + residual: max err {err:.2e} of max|y|")
    assert err < 1e-2


@pytest.mark.parametrize("outliers", [0, 5, 200])
@pytest.mark.parametrize("M,K,N", [(1, 780, 2340), (7, 2304, 780), (40, 780, 36)])
def test_generic_int8_linear_vs_oracle(M, K, N, outliers):
    """llj_g_i8_linear (LLM.int8 for K % 128 != 0: the 125M's 780 / 2304) against the oracle's
    restatement of bitsandbytes' MatMul8bitLt (parity unpinned: bitsandbytes is absent), with and
    without outlier columns, plain and with the residual add."""
    from lit_llama import _hip
    from tests.helpers import assert_bf16_close

    rng = np.random.default_rng(M + K + outliers)
    W = O.bf16_round((rng.standard_normal((N, K)) * 0.02).astype(np.float32))
    cb, scb = O.int8_quantize_weight(W)
    x = rng.standard_normal((M, K)).astype(np.float32)
    if outliers:
        x[:, rng.choice(K, outliers, replace=False)] *= 25.0
    x = O.bf16_round(x)
    res = O.bf16_round(rng.standard_normal((M, N)).astype(np.float32))
    dev = torch.device("cuda")
    xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
    cbt, scbt = torch.from_numpy(cb).to(dev), torch.from_numpy(scb).to(dev)
    ws = torch.empty(_hip.lib().llj_g_i8_ws_bytes(M, K), dtype=torch.uint8, device=dev)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    yr = torch.from_numpy(res).to(dev).to(torch.bfloat16)
    _hip.call("llj_g_i8_linear", xt.data_ptr(), K, M, K, cbt.data_ptr(), scbt.data_ptr(), 6.0, ws.data_ptr(), N,
              y.data_ptr(), N, None, 0, 0, _hip.stream())
    _hip.call("llj_g_i8_linear", xt.data_ptr(), K, M, K, cbt.data_ptr(), scbt.data_ptr(), 6.0, ws.data_ptr(), N,
              yr.data_ptr(), N, yr.data_ptr(), N, 0, _hip.stream())
    ref = O.int8_linear(x, cb, scb)
    assert_bf16_close(y.float().cpu().numpy(), ref, f"generic int8 M={M} K={K} outliers={outliers}", rel=1e-2)
    assert_bf16_close(yr.float().cpu().numpy(), O.bf16_round(res + O.bf16_round(ref)), "generic int8 resid", rel=1e-2)
    # fp32 activations (a float32 model under llm.int8): f16(x) in, the fp16 result back as fp32
    x32 = x + O.bf16_round(rng.standard_normal((M, K)).astype(np.float32) * 1e-3)  # not bf16-representable
    xt32 = torch.from_numpy(x32).to(dev)
    y32 = torch.empty(M, N, dtype=torch.float32, device=dev)
    r32 = torch.from_numpy(res).to(dev)
    _hip.call("llj_g_i8_linear", xt32.data_ptr(), K, M, K, cbt.data_ptr(), scbt.data_ptr(), 6.0, ws.data_ptr(), N,
              y32.data_ptr(), N, None, 0, 1, _hip.stream())
    yr32 = r32.clone()
    _hip.call("llj_g_i8_linear", xt32.data_ptr(), K, M, K, cbt.data_ptr(), scbt.data_ptr(), 6.0, ws.data_ptr(), N,
              yr32.data_ptr(), N, yr32.data_ptr(), N, 1, _hip.stream())
    ref32 = O.int8_linear(x32, cb, scb)
    got = y32.cpu().numpy()
    assert np.array_equal(got, got.astype(np.float16).astype(np.float32))  # fp16 values, cast back
    err = np.abs(got - ref32)
    assert (err <= 2e-3 * np.abs(ref32) + 1e-3 * np.abs(ref32).max()).all(), err.max()
    np.testing.assert_allclose(yr32.cpu().numpy(), res + got, rtol=0, atol=1e-6)
