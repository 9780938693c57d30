"""Every production kernel instantiation at the exact LLaMA-7B layer shapes (C = 4096, 32 heads
of 128, n_hidden = 11008, vocab 32000; 2 layers so the numpy oracle stays fast), for the three
--quantize modes of BASELINE.json (gptq.int4 = C2, bf16 = C1, llm.int8 = C3) at batch 1 and 8:
prefill + teacher-forced decode steps through LLaMA.forward against the oracle (bf16-emulating,
oracle/llama_np.py) on the same weights. This is where the bs=1 M == 1 instantiations
(gemv_kernel<W4, NORM, SWIGLU, 4, 4, 1, 1> etc.), the bs=8 multi-tile forms and the int8
fused launches meet an independent check at their real shapes.

Tolerance (written here), per step and row: ||logits - oracle|| / ||oracle|| < REL[mode], and
the argmax equals the oracle's wherever the oracle's top-1 / top-2 margin exceeds 4 % of
max|logit|. The oracle rounds to bf16 at the reference's points (incl. every op of the bf16
RMSNorm); what remains is fp32 summation order and 1-ulp flips that propagate through two
layers of O(1) activations: measured on MI355X 0.6-1.0e-2 for bf16 / gptq.int4 -> REL 1.5e-2.
llm.int8 re-quantizes every Linear's input to int8 per row, which turns those flips into
whole-step differences of the int8 codes (a 0.3 % input difference moves ~10 % of the codes by
one step of absmax/127): measured 2.8-3.2e-2 -> REL 5e-2. The int8 kernels themselves are held to
a tight bound on identical inputs in tests/test_kernels_gpu.py::test_int8_fused_ops_7b_shapes."""
import numpy as np
import pytest
import torch

from oracle import llama_np as O
from oracle.weights import Cfg, make_params
from tests.helpers import bf16

pytestmark = pytest.mark.gpu

C7 = Cfg(block_size=64, n_layer=2, n_head=32, n_embd=4096, vocab_size=32000)
REL = {"gptq.int4": 1.5e-2, None: 1.5e-2, "llm.int8": 5e-2}
T_PROMPT, STEPS, S = 6, 4, 32
_cache = {}


def _params():
    if "p" not in _cache:
        _cache["p"] = make_params(C7, 4096)
    _cache.setdefault("order", 0)
    return _cache["p"]


def _quant4(w):
    """Per-row min/max int4 codes (GPTQ's quantizer without error feedback), the reference's
    (N, K/2) logical quant_weight (even k in the low nibble) and bf16-exact scales / zeros."""
    xmin = np.minimum(w.min(1), 0)
    xmax = np.maximum(w.max(1), 0)
    sc = bf16(((xmax - xmin) / 15).astype(np.float32))[:, None]
    z = np.round(-xmin[:, None] / sc).astype(np.float32)
    q = np.clip(np.round(w / sc) + z, 0, 15).astype(np.uint8)
    qw = (q[:, 0::2] | (q[:, 1::2] << 4)).astype(np.uint8)
    return qw, sc, z


def _setup(mode):
    """(model, oracle) for `mode` on the shared 7B-width weights."""
    from lit_llama import LLaMA, LLaMAConfig
    from lit_llama.utils import EmptyInitOnDevice

    p = _params()
    pb = {k: bf16(v) for k, v in p.items()}
    lin, sd = {}, dict(pb)
    for k, v in p.items():
        if not k.endswith(".weight") or "wte" in k:
            continue
        name = k[:-7]
        if mode == "gptq.int4":
            qw, sc, z = _quant4(v)
            del sd[k]
            sd.update({name + ".quant_weight": qw, name + ".scales": sc, name + ".zeros": z})
            lin[name] = O.LinearSpec("colblock", qw=qw, scales=sc, zeros=z, bits=4)
        elif mode == "llm.int8":
            cb, scb = O.int8_quantize_weight(pb[k])
            lin[name] = O.LinearSpec("int8", cb=cb, scb=scb)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.bfloat16, quantization_mode=mode):
        m = LLaMA(LLaMAConfig(block_size=C7.block_size, vocab_size=C7.vocab_size, n_layer=C7.n_layer,
                              n_head=C7.n_head, n_embd=C7.n_embd))
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    orc = O.OracleLLaMA(C7, pb, linears=lin, act_bf16=True)
    return m.eval(), orc


def _gpu_steps(model, ids):
    B = ids.shape[0]
    x = torch.from_numpy(ids).cuda().long()
    model.reset_cache()
    outs = [model(x[:, :T_PROMPT], S, torch.arange(T_PROMPT).cuda())[:, -1].float()]
    for p in range(T_PROMPT, T_PROMPT + STEPS):
        outs.append(model(x[:, p:p + 1], S, torch.tensor([p]).cuda())[:, -1].float())
    model.reset_cache()
    return torch.stack(outs, 1).cpu().numpy()  # (B, steps + 1, V)


def _oracle_steps(orc, ids):
    orc.reset_cache()
    outs = [orc.forward(ids[:, :T_PROMPT], S, np.arange(T_PROMPT))[:, -1]]
    for p in range(T_PROMPT, T_PROMPT + STEPS):
        outs.append(orc.forward(ids[:, p:p + 1], S, np.array([p]))[:, -1])
    orc.reset_cache()
    return np.stack(outs, 1)


@pytest.mark.parametrize("B", [1, 2, 8])  # 2: the batched RMSNorm hand-off (nstat)
@pytest.mark.parametrize("mode", ["gptq.int4", None, "llm.int8"])
def test_7b_width_decode_vs_oracle(mode, B):
    key = ("setup", mode)
    if key not in _cache:  # one mode's model + oracle kept at a time
        for k in [k for k in _cache if k[0] == "setup"]:
            del _cache[k]
        torch.cuda.empty_cache()
        _cache[key] = _setup(mode)
    model, orc = _cache[key]
    ids = np.random.default_rng(B + 17).integers(3, C7.vocab_size, (B, T_PROMPT + STEPS + 1))
    got = _gpu_steps(model, ids)
    ref = _oracle_steps(orc, ids)
    rels = [float(np.linalg.norm(got[b, s] - ref[b, s]) / np.linalg.norm(ref[b, s]))
            for b in range(B) for s in range(STEPS + 1)]
    print(f"[7b] {mode} B={B} rel err max {max(rels):.3e} mean {np.mean(rels):.3e}")
    for b in range(B):
        for s in range(STEPS + 1):
            g, r = got[b, s], ref[b, s]
            rel = float(np.linalg.norm(g - r) / np.linalg.norm(r))
            assert rel < REL[mode], f"{mode} B={B} row {b} step {s}: rel err {rel:.3e}"
            top2 = np.sort(r)[-2:]
            if top2[1] - top2[0] > 4e-2 * np.abs(r).max():
                assert int(g.argmax()) == int(r.argmax()), f"{mode} B={B} row {b} step {s}: argmax"
