"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE implementation.

Runs only in the build container, where /root/reference (if001/lit-llama-ja, read-only)
is mounted. The reference never travels: only the .npz inputs/outputs written here are
committed, and the tests regenerate the (seeded) weights through oracle/weights.py.

The reference imports `lightning` (generate.py:7, lit_llama/utils.py:13) only for the
Fabric CLI plumbing and for isinstance checks in checkpoint-saving helpers, none of which
is on the path exercised here. `lightning` is not installed in this image, so a
placeholder module with dummy names is put in sys.modules before importing; it provides
no computation. bitsandbytes is absent, so Linear8bitLt is not defined by the reference
here and no llm.int8 fixture can be produced (int8 parity is unpinned).

Usage:  python tests/golden/make_golden.py   (≈1–2 min on 8 CPUs)
"""
from __future__ import annotations

import contextlib
import io
import os
import sys
import types
from pathlib import Path

os.environ.setdefault("TRITON_INTERPRET", "1")  # run the Triton int4 kernel body on CPU

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REF))

# --- placeholder for the absent `lightning` package (no computation behind it) -------
_l = types.ModuleType("lightning")
_lf = types.ModuleType("lightning.fabric")
_lfs = types.ModuleType("lightning.fabric.strategies")


class _Dummy:  # isinstance targets only
    pass


_lfs.DeepSpeedStrategy = _Dummy
_lfs.FSDPStrategy = _Dummy
_l.fabric = _lf
_lf.strategies = _lfs
_l.Fabric = _Dummy
_l.seed_everything = lambda s: torch.manual_seed(s)
sys.modules.update({"lightning": _l, "lightning.fabric": _lf, "lightning.fabric.strategies": _lfs})

from lit_llama.model import LLaMA, LLaMAConfig, RMSNorm, apply_rope, build_rope_cache  # noqa: E402
from lit_llama import quantization as rq  # noqa: E402
import generate as rgen  # noqa: E402
from quantize.gptq import llama_blockwise_quantization  # noqa: E402

from oracle.weights import Cfg, make_params, make_prompt, ref_init_params  # noqa: E402

torch.set_num_threads(8)
TOPK = 5


def ref_model(cfg: Cfg, params: dict, dtype=torch.float32) -> LLaMA:
    rc = LLaMAConfig(block_size=cfg.block_size, vocab_size=cfg.vocab_size, n_layer=cfg.n_layer,
                     n_head=cfg.n_head, n_embd=cfg.n_embd)
    m = LLaMA(rc)
    sd = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
    m.load_state_dict(sd)
    return m.to(dtype).eval()


@torch.no_grad()
def greedy_trace(model, prompt: np.ndarray, n_new: int, max_seq_length=None, eos_id=None):
    """Runs the reference generate() with top_k=1 (greedy) and records per-step logits."""
    steps = []
    orig_forward = model.forward

    def spy(idx, msl=None, input_pos=None):
        out = orig_forward(idx, msl, input_pos)
        steps.append(out[0, -1].float().clone())
        return out

    model.forward = spy
    try:
        out = rgen.generate(model, torch.from_numpy(prompt.astype(np.int32)), n_new,
                            max_seq_length=max_seq_length, temperature=1.0, top_k=1, eos_id=eos_id)
    finally:
        model.forward = orig_forward
        model.reset_cache()
    L = torch.stack(steps)  # (n_steps, V)
    v, i = torch.topk(L, TOPK, dim=-1)
    return out.numpy().astype(np.int32), L.numpy(), v.numpy(), i.numpy().astype(np.int32)


def save(name: str, **arrays):
    path = HERE / f"{name}.npz"
    np.savez_compressed(path, **arrays)
    print(f"wrote {path.relative_to(REPO)} ({path.stat().st_size/1024:.0f} KiB)")


# -------------------------------------------------------------------------------------
def gen_ops():
    torch.manual_seed(1)
    out = {}
    for hs in (64, 128):
        c = build_rope_cache(seq_len=32, n_elem=hs, dtype=torch.int32, device=torch.device("cpu"))
        out[f"rope_cache_{hs}"] = c.numpy()
        x = torch.randn(2, 6, 3, hs)
        out[f"rope_x_{hs}"] = x.numpy()
        out[f"rope_y_{hs}"] = apply_rope(x, c[:6]).numpy()
        # decode-style: rope rows gathered at arbitrary positions (model.py:101-102)
        pos = torch.tensor([0, 5, 17, 31])
        xr = torch.randn(4, 1, 3, hs)
        out[f"rope_pos_{hs}"] = pos.numpy()
        out[f"rope_xd_{hs}"] = xr.numpy()
        out[f"rope_yd_{hs}"] = torch.cat([apply_rope(xr[j:j + 1], c.index_select(0, pos[j:j + 1]))
                                          for j in range(4)]).numpy()
    for C in (256, 4096):
        x = torch.randn(3, 5, C) * 3
        n = RMSNorm(C)
        with torch.no_grad():
            n.scale.copy_(torch.rand(C) + 0.5)
        out[f"rms_x_{C}"] = x.numpy()
        out[f"rms_scale_{C}"] = n.scale.detach().numpy()
        out[f"rms_y_{C}"] = n(x).detach().numpy()
        nb = RMSNorm(C).to(torch.bfloat16)
        with torch.no_grad():
            nb.scale.copy_(n.scale.to(torch.bfloat16))
        out[f"rms_ybf16_{C}"] = nb(x.to(torch.bfloat16)).float().detach().numpy()
    save("ops", **out)


def gen_colblock():
    """ColBlockQuantizedLinear pack/get_weight/forward + the Triton kernel body (interpreted)."""
    torch.manual_seed(2)
    out = {}
    for bits in (4, 8):
        N, K = 160, 384
        lin = rq.ColBlockQuantizedLinear(K, N, False, bits=bits, tile_cols=-1)
        W = torch.randn(N, K) * 0.05
        maxq = 2 ** bits - 1
        xmin = torch.minimum(W.min(1)[0], torch.zeros(N))
        xmax = torch.maximum(W.max(1)[0], torch.zeros(N))
        scale = (xmax - xmin) / maxq
        zero = torch.round(-xmin / scale)
        lin.scales.copy_(scale[:, None])
        lin.zeros.copy_(zero[:, None])
        # pack the GPTQ-style reconstruction scale*(q-zero) exactly as GPTQQuantizer.quantize
        # feeds pack_weight (quantization.py:603-614)
        q = torch.clamp(torch.round(W / scale[:, None]) + zero[:, None], 0, maxq)
        Wrec = scale[:, None] * (q - zero[:, None])
        lin.pack_weight(Wrec)
        out[f"b{bits}_qw"] = lin.quant_weight.contiguous().numpy()  # logical (N, K*bits/8)
        out[f"b{bits}_scales"] = lin.scales.numpy()
        out[f"b{bits}_zeros"] = lin.zeros.numpy()
        out[f"b{bits}_wdeq"] = lin.get_weight(torch.float).numpy()
        out[f"b{bits}_wdeq_bf16"] = lin.get_weight(torch.bfloat16).float().numpy()
        for M in (1, 3, 8):
            x = torch.randn(M, K)
            out[f"b{bits}_x{M}"] = x.numpy()
            out[f"b{bits}_y{M}"] = lin(x).detach().numpy()
            # bf16 CPU fallback path (what runs off-GPU on a bf16 model)
            lb = rq.ColBlockQuantizedLinear(K, N, False, bits=bits, tile_cols=-1)
            lb.load_state_dict(lin.state_dict())
            lb.scales = lb.scales.to(torch.bfloat16)
            lb.zeros = lb.zeros.to(torch.bfloat16)
            out[f"b{bits}_ybf16_{M}"] = lb(x.to(torch.bfloat16)).float().detach().numpy()
        if bits == 4 and rq.triton is not None:
            # Triton GPU-path semantics, body run by the interpreter on CPU
            try:
                for M in (1, 3, 8):
                    x = torch.from_numpy(out[f"b4_x{M}"])
                    w = lin.quant_weight.t().contiguous()  # (K/2, N)
                    c = torch.empty(M, N)
                    grid = (triton_cdiv(M, 32) * triton_cdiv(N, 64),)
                    rq.linear_kernel_4bit_weight.fn[grid](
                        x, w, c, lin.scales.contiguous(), lin.zeros.contiguous(), M, N, K,
                        x.stride(0), x.stride(1), w.stride(0), w.stride(1), c.stride(0), c.stride(1),
                        BLOCK_SIZE_M=32, BLOCK_SIZE_N=64, BLOCK_SIZE_K=32, GROUP_SIZE_M=8)
                    out[f"b4_ytriton{M}"] = c.numpy()
            except Exception as e:  # interpreter unavailable: recorded, fixture still valid
                print("triton interpreter run skipped:", repr(e)[:200])
    save("colblock", **out)


def triton_cdiv(a, b):
    return (a + b - 1) // b


def gen_tiny():
    """C0: LLaMAConfig(block_size=128, n_layer=2, n_head=4, n_embd=256), V=32000."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=32000)
    seed = 1234
    params = make_params(cfg, seed)
    prompt = make_prompt(8, cfg.vocab_size, seed)
    out = {"seed": np.int64(seed), "prompt": prompt}
    for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        m = ref_model(cfg, params, dt)
        ids, L, v, i = greedy_trace(m, prompt, 32)
        out[f"{tag}_ids"] = ids
        out[f"{tag}_top_v"] = v
        out[f"{tag}_top_i"] = i
        out[f"{tag}_logits_step0"] = L[0]
        out[f"{tag}_logits_step1"] = L[1]
    # full prefill logits (all 8 rows) through the no-cache path (input_pos=None)
    m = ref_model(cfg, params)
    with torch.no_grad():
        out["fp32_prefill_nocache"] = m(torch.from_numpy(prompt[None]).long()).numpy()[0]
    save("tiny_c0", **out)


def gen_int4_gptq():
    """GPTQ-packed int4 model (reference quantize/gptq.py) + its greedy trace."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=2048)
    seed = 4321
    params = make_params(cfg, seed)
    m = ref_model(cfg, params)
    g = torch.Generator().manual_seed(seed)
    calib = torch.randint(3, cfg.vocab_size, (4, cfg.block_size), generator=g)  # gptq.py:90 needs T == block_size
    with contextlib.redirect_stdout(io.StringIO()):
        llama_blockwise_quantization(m, calib, "cpu", bits=4)
    sd = m.state_dict()
    out = {"seed": np.int64(seed)}
    for k, v in sd.items():
        if k.endswith(("quant_weight", "scales", "zeros")):
            out["sd/" + k] = v.contiguous().numpy()
    prompt = make_prompt(6, cfg.vocab_size, seed)
    out["prompt"] = prompt
    m.eval()
    ids, L, v, i = greedy_trace(m, prompt, 24)
    out.update(fp32_ids=ids, fp32_top_v=v, fp32_top_i=i, fp32_logits_step0=L[0], fp32_logits_step5=L[5])
    mb = m.to(torch.bfloat16)
    ids, L, v, i = greedy_trace(mb, prompt, 24)
    out.update(bf16_ids=ids, bf16_top_v=v, bf16_top_i=i, bf16_logits_step0=L[0])
    save("int4_gptq", **out)


def gen_gptq():
    """GPTQQuantizer (quantization.py:424-614) on single Linears: inputs W and calibration
    activations X, the reference's accumulated Hessian H, and its packed outputs. Cases: one
    128-column block (with a dead input column), three blocks, bits=8."""
    out = {}
    cases = {"a": (96, 128, 4, 11), "b": (160, 384, 4, 12), "c": (64, 256, 8, 13)}
    for tag, (N, K, bits, seed) in cases.items():
        rng = np.random.default_rng(seed)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        W[:, :8] *= 4.0  # a few wide columns (act-order has something to sort)
        X = rng.standard_normal((4, 32, K)).astype(np.float32) * rng.uniform(0.2, 2.0, K).astype(np.float32)
        if tag == "a":
            X[..., 5] = 0.0  # dead column: diag(H) == 0 (quantization.py:544-546)
        lin = torch.nn.Linear(K, N, bias=False)
        lin.weight.data = torch.from_numpy(W.copy())
        gq = rq.GPTQQuantizer(lin, bits=bits, groupsize=-1, actorder=True)
        h = lin.register_forward_hook(gq.collect_input_stats)
        with torch.no_grad():
            for j in range(X.shape[0]):  # one sample per call, as quantize/gptq.py:96-104
                lin(torch.from_numpy(X[j:j + 1]))
        h.remove()
        H = gq.H.clone().numpy()
        qm, err = gq.quantize()
        out.update({f"{tag}_W": W, f"{tag}_X": X, f"{tag}_H": H, f"{tag}_bits": np.int64(bits),
                    f"{tag}_quant_weight": qm.quant_weight.contiguous().numpy(),
                    f"{tag}_scales": qm.scales.numpy().reshape(-1), f"{tag}_zeros": qm.zeros.numpy().reshape(-1),
                    f"{tag}_error": np.float64(err)})
    save("gptq", **out)


def gen_gptq_opts():
    """GPTQQuantizer (quantization.py:424-614) with the constructor options quantize/gptq.py leaves at
    their defaults: sym=True (find_params_weight 488-501: symmetric range, zero (maxq + 1) / 2),
    perchannel=False (479-482, 503-506: one (scale, zero) for the whole matrix, repeated per row) and
    blocksizes 64 / 32 (557: the lazy-batch block of the column loop). Same record as gen_gptq plus
    the options."""
    out = {}
    cases = {"sym": (96, 256, 4, 128, True, True, True, 31), "pt": (64, 256, 4, 128, False, False, True, 32),
             "b64": (80, 384, 4, 64, True, False, True, 33), "b32": (64, 256, 8, 32, True, True, False, 34),
             "b16": (48, 128, 4, 16, False, True, False, 35)}
    for tag, (N, K, bits, bs, perch, sym, act, seed) in cases.items():
        rng = np.random.default_rng(seed)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        W[:, :8] *= 4.0
        W[:16] += 0.02  # rows with a one-signed range (the symmetric rule's xmin >= 0 branch)
        W[:4] = np.abs(W[:4])
        X = rng.standard_normal((4, 32, K)).astype(np.float32) * rng.uniform(0.2, 2.0, K).astype(np.float32)
        lin = torch.nn.Linear(K, N, bias=False)
        lin.weight.data = torch.from_numpy(W.copy())
        gq = rq.GPTQQuantizer(lin, bits=bits, perchannel=perch, sym=sym, blocksize=bs, groupsize=-1, actorder=act)
        h = lin.register_forward_hook(gq.collect_input_stats)
        with torch.no_grad():
            for j in range(X.shape[0]):
                lin(torch.from_numpy(X[j:j + 1]))
        h.remove()
        H = gq.H.clone().numpy()
        qm, err = gq.quantize()
        out.update({f"{tag}_W": W, f"{tag}_X": X, f"{tag}_H": H, f"{tag}_bits": np.int64(bits),
                    f"{tag}_opts": np.array([bs, int(perch), int(sym), int(act)], np.int64),
                    f"{tag}_quant_weight": qm.quant_weight.contiguous().numpy(),
                    f"{tag}_scales": qm.scales.numpy().reshape(-1), f"{tag}_zeros": qm.zeros.numpy().reshape(-1),
                    f"{tag}_error": np.float64(err)})
    save("gptq_opts", **out)


def gen_gptq_grouped():
    """Grouped ColBlockQuantizedLinear (tile_cols = g; pack_weight / get_weight / forward =
    get_weight + F.linear, quantization.py:374-421) with per-group (scale, zero) from the
    reference's own GPTQQuantizer.find_params_weight on each group's columns. Cases: g = 128 over
    K = 384 (3 groups), g = 256 over K = 640 (a ragged last group of 128 columns).
    The reference's grouped GPTQ column loop itself raises (quantization.py:576 assigns the
    (N, 1) scale from find_params_weight into the (N,) column scales[:, j]: "expand ... the number
    of sizes provided (1) must be greater or equal to the number of dimensions"), so the grouped
    PRODUCER has no reference output: it is checked against oracle/gptq_np.py only (parity
    unpinned), on the W / X recorded here."""
    out = {}
    cases = {"g1": (96, 384, 128, 21), "g2": (64, 640, 256, 22)}
    for tag, (N, K, g, seed) in cases.items():
        rng = np.random.default_rng(seed)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        W[:, :8] *= 4.0
        W[:, K // 2: K // 2 + 8] *= 3.0  # wide columns inside a later group
        X = rng.standard_normal((4, 32, K)).astype(np.float32) * rng.uniform(0.2, 2.0, K).astype(np.float32)
        lin = torch.nn.Linear(K, N, bias=False)
        lin.weight.data = torch.from_numpy(W.copy())
        gq = rq.GPTQQuantizer(lin, bits=4, groupsize=g, actorder=False)
        G = (K + g - 1) // g
        qm = rq.ColBlockQuantizedLinear(K, N, False, bits=4, tile_cols=g)
        Wt = torch.from_numpy(W.copy())
        Wrec = torch.empty_like(Wt)
        for j in range(G):
            sl = slice(j * g, min(K, (j + 1) * g))
            sc, zr = gq.find_params_weight(Wt[:, sl])
            qm.scales[:, j] = sc[:, 0]
            qm.zeros[:, j] = zr[:, 0]
            q = torch.clamp(torch.round(Wt[:, sl] / sc) + zr, 0, 15)
            Wrec[:, sl] = sc * (q - zr)
        qm.pack_weight(Wrec)
        out.update({f"{tag}_W": W, f"{tag}_X": X, f"{tag}_g": np.int64(g),
                    f"{tag}_quant_weight": qm.quant_weight.contiguous().numpy(),
                    f"{tag}_scales": qm.scales.numpy(), f"{tag}_zeros": qm.zeros.numpy(),
                    f"{tag}_wdeq": qm.get_weight(torch.float).numpy(),
                    f"{tag}_wdeq_bf16": qm.get_weight(torch.bfloat16).float().numpy()})
        for M in (1, 5):
            x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
            with torch.no_grad():
                out[f"{tag}_x{M}"] = x.numpy()
                out[f"{tag}_y{M}"] = qm(x).numpy()
        try:
            gq.quantize()  # recorded: the reference's grouped column loop raises
            out[f"{tag}_ref_quantize_raises"] = np.int64(0)
        except RuntimeError:
            out[f"{tag}_ref_quantize_raises"] = np.int64(1)
    save("gptq_grouped", **out)

def gen_hf_convert():
    """The reference's scripts/convert_hf_checkpoint.py on a tiny synthetic HF LLaMA checkpoint
    (two .bin shards, layer 1's q / k / v split across them, rotary inv_freq buffers), written to
    a temporary directory; the fixture holds the HF tensors and the converted lit-llama tensors."""
    import json
    import tempfile

    from lit_llama import model as rmodel
    from scripts.convert_hf_checkpoint import convert_hf_checkpoint

    rmodel.llama_configs["tinyhf"] = dict(n_layer=2, n_head=4, n_embd=64, vocab_size=128)
    C, H, V, L = 64, 256, 128, 2
    rng = np.random.default_rng(77)
    t = lambda *sh: torch.from_numpy(rng.standard_normal(sh).astype(np.float32))  # noqa: E731
    hf = {"model.embed_tokens.weight": t(V, C), "model.norm.weight": t(C), "lm_head.weight": t(V, C)}
    for i in range(L):
        p = f"model.layers.{i}."
        hf.update({p + "self_attn.q_proj.weight": t(C, C), p + "self_attn.k_proj.weight": t(C, C),
                   p + "self_attn.v_proj.weight": t(C, C), p + "self_attn.o_proj.weight": t(C, C),
                   p + "self_attn.rotary_emb.inv_freq": t(C // 8), p + "mlp.gate_proj.weight": t(H, C),
                   p + "mlp.up_proj.weight": t(H, C), p + "mlp.down_proj.weight": t(C, H),
                   p + "input_layernorm.weight": t(C), p + "post_attention_layernorm.weight": t(C)})
    shard1 = {k: v for k, v in hf.items() if "layers.1." not in k or "q_proj" in k}
    shard2 = {k: v for k, v in hf.items() if k not in shard1}
    with tempfile.TemporaryDirectory() as td:
        ck, out = Path(td) / "hf" / "tinyhf", Path(td) / "lit" / "tinyhf"
        ck.mkdir(parents=True)
        (ck / "tokenizer.model").write_bytes(b"placeholder")
        names = {"pytorch_model-00001-of-00002.bin": shard1, "pytorch_model-00002-of-00002.bin": shard2}
        for fn, sd in names.items():
            torch.save(sd, ck / fn)
        wm = {k: fn for fn, sd in names.items() for k in sd}
        (ck / "pytorch_model.bin.index.json").write_text(json.dumps({"metadata": {}, "weight_map": wm}))
        with contextlib.redirect_stdout(io.StringIO()):
            convert_hf_checkpoint(output_dir=out, checkpoint_dir=ck, model_size="tinyhf", dtype="float32")
        from lit_llama.utils import lazy_load  # the reference's own reader of its incremental_save format
        with lazy_load(out / "lit-llama.pth") as sd:
            lit = {k: v._load_tensor() for k, v in sd.items()}
    arrays = {"hf/" + k: v.numpy() for k, v in hf.items()}
    arrays.update({"lit/" + k: v.numpy() for k, v in lit.items()})
    arrays["shard1_keys"] = np.array(sorted(shard1))
    save("hf_convert", **arrays)


def gen_meta_convert():
    """The reference's scripts/convert_checkpoint.py (meta_weights_for_nano_model) on a tiny
    synthetic Meta checkpoint split over two model-parallel files."""
    import tempfile

    from scripts.convert_checkpoint import meta_weights_for_nano_model

    C, H, V, L, n = 64, 256, 128, 2, 2
    rng = np.random.default_rng(78)
    t = lambda *sh: torch.from_numpy(rng.standard_normal(sh).astype(np.float32))  # noqa: E731
    parts = []
    for _ in range(n):
        sd = {"tok_embeddings.weight": t(V, C // n), "output.weight": t(V // n, C), "norm.weight": t(C)}
        for i in range(L):
            p = f"layers.{i}."
            sd.update({p + "attention.wq.weight": t(C // n, C), p + "attention.wk.weight": t(C // n, C),
                       p + "attention.wv.weight": t(C // n, C), p + "attention.wo.weight": t(C, C // n),
                       p + "feed_forward.w1.weight": t(H // n, C), p + "feed_forward.w2.weight": t(C, H // n),
                       p + "feed_forward.w3.weight": t(H // n, C), p + "attention_norm.weight": t(C),
                       p + "ffn_norm.weight": t(C)})
        parts.append(sd)
    with tempfile.TemporaryDirectory() as td:
        ck = Path(td) / "llama" / "tinymeta"
        ck.mkdir(parents=True)
        (ck.parent / "tokenizer.model").write_bytes(b"placeholder")
        for r, sd in enumerate(parts):
            torch.save(sd, ck / f"consolidated.{r:02d}.pth")
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            meta_weights_for_nano_model(output_dir=Path(td) / "lit", checkpoint_dir=Path(td) / "llama",
                                        model_size="tinymeta")
        lit = torch.load(Path(td) / "lit" / "tinymeta" / "lit-llama.pth", map_location="cpu", weights_only=True)
    arrays = {f"meta{r}/" + k: v.numpy() for r, sd in enumerate(parts) for k, v in sd.items()}
    arrays.update({"lit/" + k: v.numpy() for k, v in lit.items()})
    save("meta_convert", **arrays)


def gen_kv_roll():
    """Sliding-window KV roll (model.py:221-225), as tests/test_generate.py:46 exercises."""
    cfg = Cfg(block_size=128, n_layer=1, n_head=4, n_embd=256, vocab_size=512)
    seed = 99
    params = make_params(cfg, seed)
    prompt = make_prompt(5, cfg.vocab_size, seed)
    m = ref_model(cfg, params)
    steps = []
    orig_forward = m.forward
    caches = {}

    def spy(idx, msl=None, input_pos=None):
        o = orig_forward(idx, msl, input_pos)
        steps.append(o[0, -1].clone())
        caches["k"] = m.kv_caches[0][0].clone()
        caches["v"] = m.kv_caches[0][1].clone()
        return o

    m.forward = spy
    with torch.no_grad():
        ids = rgen.generate(m, torch.from_numpy(prompt), 20, max_seq_length=10, top_k=1)
    L = torch.stack(steps)
    v, i = torch.topk(L, TOPK, -1)
    save("kv_roll", seed=np.int64(seed), prompt=prompt, ids=ids.numpy().astype(np.int32),
         top_v=v.numpy(), top_i=i.numpy().astype(np.int32),
         k_cache=caches["k"].numpy(), v_cache=caches["v"].numpy())


@torch.no_grad()
def gen_batch():
    """bs=8 batched prefill+decode through LLaMA.forward (the reference model supports B>1)."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=2048)
    seed = 777
    params = make_params(cfg, seed)
    B, T, steps, S = 8, 6, 6, 16
    prompts = make_prompt(T, cfg.vocab_size, seed, batch=B)
    m = ref_model(cfg, params)
    idx = torch.from_numpy(prompts).long()
    pos = torch.arange(T)
    tops_v, tops_i, ids = [], [], []
    x = idx
    for s in range(steps):
        L = m(x, S, pos)[:, -1]
        v, i = torch.topk(L, TOPK, -1)
        tops_v.append(v.numpy()); tops_i.append(i.numpy())
        nxt = L.argmax(-1)
        ids.append(nxt.numpy())
        x = nxt[:, None]
        pos = pos[-1:] + 1
    m.reset_cache()
    # per-row check against B=1 runs (documents that batching is exact up to fp rounding)
    for b in range(B):
        pb = torch.arange(T)
        xb = idx[b:b + 1]
        for s in range(steps):
            Lb = m(xb, S, pb)[:, -1]
            assert int(Lb.argmax()) == int(ids[s][b])
            xb = Lb.argmax(-1)[:, None]
            pb = pb[-1:] + 1
        m.reset_cache()
    save("batch8", seed=np.int64(seed), prompts=prompts, ids=np.stack(ids).T.astype(np.int32),
         top_v=np.stack(tops_v), top_i=np.stack(tops_i).astype(np.int32))


def gen_eos():
    """EOS stop: generate() returns idx[:input_pos], i.e. WITHOUT the EOS token (generate.py:86-87)."""
    cfg = Cfg(block_size=64, n_layer=1, n_head=4, n_embd=256, vocab_size=512)
    seed = 5
    params = make_params(cfg, seed)
    prompt = make_prompt(4, cfg.vocab_size, seed)
    m = ref_model(cfg, params)
    full, *_ = greedy_trace(m, prompt, 12)
    eos = int(full[4 + 5])  # the 6th generated token
    first = int(np.nonzero(full[4:] == eos)[0][0])
    stopped, *_ = greedy_trace(m, prompt, 12, eos_id=eos)
    save("eos", seed=np.int64(seed), prompt=prompt, full=full, eos_id=np.int64(eos),
         first_eos_step=np.int64(first), stopped=stopped)


def gen_sampled():
    """Sampled decoding (generate.py:66-74: temperature 0.8, top_k 50) through the reference's own
    generate() on a bf16 model, with torch.multinomial replaced by an inverse-CDF draw at recorded
    uniforms (the first index whose running sum of the probs it is handed exceeds u * sum). The
    fixture keeps the uniforms, the probability rows the reference computed, and the ids."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=2048)
    seed = 4242
    params = make_params(cfg, seed)
    prompt = make_prompt(8, cfg.vocab_size, seed)
    m = ref_model(cfg, params, dtype=torch.bfloat16)
    rng = np.random.default_rng(seed)
    us, probs = [], []

    def inv_cdf(p, num_samples=1):
        u = float(rng.random())
        us.append(u)
        probs.append(p.float().numpy().copy())
        c = torch.cumsum(p.double(), -1)
        i = int(torch.nonzero(c > u * c[-1])[0, 0])
        return torch.tensor([i])

    orig = torch.multinomial
    torch.multinomial = inv_cdf
    try:
        with torch.no_grad():
            out = rgen.generate(m, torch.from_numpy(prompt.astype(np.int32)), 16, temperature=0.8, top_k=50)
    finally:
        torch.multinomial = orig
    save("sampled", seed=np.int64(seed), prompt=prompt, ids=out.numpy().astype(np.int32),
         u=np.array(us, np.float32), probs=np.stack(probs).astype(np.float32))


def gen_sampled_fp32():
    """The same sampled decoding (temperature 0.8, top_k 50, recorded uniforms) on the reference's
    float32 model -- generate.py's own defaults (top_k 200, temperature 0.8) run fp32 on a host without
    bf16 (generate.py:97-98, 121): logits / temperature, topk threshold, softmax and the draw in fp32.
    Keeps the uniforms, the fp32 probability rows and the ids."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=2048)
    seed = 4243
    params = make_params(cfg, seed)
    prompt = make_prompt(8, cfg.vocab_size, seed)
    m = ref_model(cfg, params, dtype=torch.float32)
    rng = np.random.default_rng(seed)
    us, probs = [], []

    def inv_cdf(p, num_samples=1):
        u = float(rng.random())
        us.append(u)
        probs.append(p.float().numpy().copy())
        c = torch.cumsum(p.double(), -1)
        i = int(torch.nonzero(c > u * c[-1])[0, 0])
        return torch.tensor([i])

    orig = torch.multinomial
    torch.multinomial = inv_cdf
    try:
        with torch.no_grad():
            out = rgen.generate(m, torch.from_numpy(prompt.astype(np.int32)), 16, temperature=0.8, top_k=50)
    finally:
        torch.multinomial = orig
    save("sampled_fp32", seed=np.int64(seed), prompt=prompt, ids=out.numpy().astype(np.int32),
         u=np.array(us, np.float32), probs=np.stack(probs).astype(np.float32))


def gen_ppl():
    """The reference's perplexity loop (evaluate/full.py:114-128) on the tiny C0 model in fp32: a
    300-token stream cut into block_size (128) windows, logits[:-1] scored against inp[1:] with a
    summed cross entropy."""
    cfg = Cfg(block_size=128, n_layer=2, n_head=4, n_embd=256, vocab_size=32000)
    seed = 31
    m = ref_model(cfg, make_params(cfg, seed))
    tokens = make_prompt(300, cfg.vocab_size, seed)[None].astype(np.int64)
    enc = torch.from_numpy(tokens)
    nlls, toks, per = 0.0, 0, []
    with torch.inference_mode():
        for i in range(0, enc.shape[1], cfg.block_size):
            inp = enc[:, i:i + cfg.block_size]
            logits = m(inp)[0]
            nll = torch.nn.functional.cross_entropy(logits[:-1], inp[0, 1:].to(dtype=torch.long), reduction="sum")
            toks += inp.size(1) - 1
            nlls += nll.item()
            per.append(nll.item())
    save("ppl", seed=np.int64(seed), tokens=tokens, nll_per_window=np.array(per), toks=np.int64(toks),
         ppl=np.float64(np.exp(nlls / toks)))


def gen_bf16_init():
    """The reference's bf16 acceptance test (tests/test_model.py:103-131) at a shape the gfx950
    kernels take: an fp32 LLaMA at the reference's init scale (ref_init_params = _init_weights'
    N(0, 0.02/sqrt(2 n_layer))), 16 layers, batch 3, a full block of 64 tokens through the no-cache
    forward; the expected fp32 logits of every position. The test loads the same weights into a
    bf16 model on the GPU and applies the reference's criterion assert_close(atol=5e-3, rtol=1e-3).
    Differences from the reference test: n_embd 256 / n_head 4 (hs 64) instead of 32 / 16 (hs 2),
    vocab 512 instead of 32000 (fixture size), numpy instead of torch RNG for the weights."""
    cfg = Cfg(block_size=64, n_layer=16, n_head=4, n_embd=256, vocab_size=512)
    seed = 103
    params = ref_init_params(cfg, seed)
    m = ref_model(cfg, params)
    rng = np.random.default_rng(seed)
    tokens = rng.integers(0, cfg.vocab_size, size=(3, cfg.block_size)).astype(np.int64)
    with torch.no_grad():
        expected = m(torch.from_numpy(tokens)).float().numpy()
    save("bf16_init", seed=np.int64(seed), tokens=tokens, expected=expected.astype(np.float32))


def gen_ref_ckpt():
    """A lit-llama.pth exactly as the reference writes it: its scripts/convert_hf_checkpoint.py
    (which streams through its incremental_save, protocol 5, lit_llama/utils.py:492-531) run with
    dtype="bfloat16" on a synthetic HF checkpoint of a shape the gfx950 kernels take (n_embd 128,
    2 heads of 64, n_hidden 512, vocab 256, 2 layers; O(1) activations like oracle.weights). The
    .pth file itself is the fixture (ref_lit_llama_bf16.pth, data written by the reference), with
    digests of the tensors the reference's own lazy_load reads back from it (ref_ckpt.npz)."""
    import json
    import shutil
    import tempfile

    from lit_llama import model as rmodel
    from scripts.convert_hf_checkpoint import convert_hf_checkpoint

    C, nh, H, V, L = 128, 2, 512, 256, 2
    rmodel.llama_configs["tinyref"] = dict(n_layer=L, n_head=nh, n_embd=C, vocab_size=V, block_size=64)
    rng = np.random.default_rng(79)
    t = lambda *sh: torch.from_numpy((rng.standard_normal(sh) / np.sqrt(sh[-1])).astype(np.float32))  # noqa: E731
    u = lambda n: torch.from_numpy(rng.uniform(0.5, 1.5, n).astype(np.float32))  # noqa: E731
    hf = {"model.embed_tokens.weight": torch.from_numpy(rng.standard_normal((V, C)).astype(np.float32)),
          "model.norm.weight": u(C), "lm_head.weight": t(V, C) * 2}
    for i in range(L):
        p = f"model.layers.{i}."
        hf.update({p + "self_attn.q_proj.weight": t(C, C), p + "self_attn.k_proj.weight": t(C, C),
                   p + "self_attn.v_proj.weight": t(C, C), p + "self_attn.o_proj.weight": t(C, C),
                   p + "mlp.gate_proj.weight": t(H, C), p + "mlp.up_proj.weight": t(H, C),
                   p + "mlp.down_proj.weight": t(C, H), p + "input_layernorm.weight": u(C),
                   p + "post_attention_layernorm.weight": u(C)})
    with tempfile.TemporaryDirectory() as td:
        ck, out = Path(td) / "hf" / "tinyref", Path(td) / "lit" / "tinyref"
        ck.mkdir(parents=True)
        (ck / "tokenizer.model").write_bytes(b"placeholder")
        torch.save(hf, ck / "pytorch_model-00001-of-00001.bin")
        wm = {k: "pytorch_model-00001-of-00001.bin" for k in hf}
        (ck / "pytorch_model.bin.index.json").write_text(json.dumps({"metadata": {}, "weight_map": wm}))
        with contextlib.redirect_stdout(io.StringIO()):
            convert_hf_checkpoint(output_dir=out, checkpoint_dir=ck, model_size="tinyref", dtype="bfloat16")
        from lit_llama.utils import lazy_load  # the reference's own reader of its incremental_save format
        with lazy_load(out / "lit-llama.pth") as sd:
            lit = {k: v._load_tensor() for k, v in sd.items()}
        shutil.copy(out / "lit-llama.pth", HERE / "ref_lit_llama_bf16.pth")
        print(f"wrote tests/golden/ref_lit_llama_bf16.pth ({(HERE / 'ref_lit_llama_bf16.pth').stat().st_size} B)")
    import hashlib

    # per tensor: sha256 of the bytes the reference's lazy_load returns (C order), shape, dtype
    arrays = {}
    for k, v in lit.items():
        b = v.contiguous().view(torch.int16).numpy().tobytes()
        arrays["sha/" + k] = np.array(hashlib.sha256(b).hexdigest())
        arrays["shape/" + k] = np.array(v.shape, np.int64)
        arrays["dtype/" + k] = np.array(str(v.dtype))
    arrays["config"] = np.array([C, nh, V, L, 64], np.int64)
    save("ref_ckpt", **arrays)


if __name__ == "__main__":
    which = sys.argv[1:] or ["ops", "colblock", "tiny", "int4_gptq", "kv_roll", "batch", "eos", "gptq", "hf_convert",
                             "meta_convert", "bf16_init", "sampled", "sampled_fp32", "ppl", "gptq_grouped", "ref_ckpt", "gptq_opts"]
    for w in which:
        globals()[f"gen_{w}"]()
