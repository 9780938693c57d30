"""Whole-model GPTQ driver (reference quantize/gptq.py:36-148, `llama_blockwise_quantization`):
blocks in order, each Linear quantized from the inputs it sees with its predecessors already
quantized, then ln_f and lm_head. The quantizer is lit_llama.quantization.GPTQQuantizer (HIP
column loop + device GEMM / Cholesky). The calibration forward of a block (`calib_block`) runs
the model's own kernels where the decode path has them (RMSNorm: llj_rmsnorm; the Linears through
their modules, so the forward hooks fire: plain nn.Linear before quantization, the HIP
ColBlockQuantizedLinear after) and torch's scaled_dot_product_attention for the T x T causal
attention of a calibration window (prefill attention is SURVEY §8f row 3, not built). Activations
are bf16 like the decode path (the reference's CPU runs calibrate in fp32)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from lit_llama.model import apply_rope
from lit_llama.quantization import GPTQQuantizer

SUBMODULES = ["attn.c_attn", "attn.c_proj", "mlp.c_fc1", "mlp.c_fc2", "mlp.c_proj"]  # reference 63-69


def calib_block(block, x: torch.Tensor, rope: torch.Tensor) -> torch.Tensor:
    """Block.forward without a KV cache (reference model.py:162-175, 192-242) for one window
    x (1, T, C) bf16, calling every Linear through its module."""
    _, T, C = x.shape
    nh = block.attn.n_head
    hs = C // nh
    h = block.rms_1(x)
    q, k, v = block.attn.c_attn(h).split(C, dim=2)
    q = apply_rope(q.reshape(1, T, nh, hs), rope).transpose(1, 2)
    k = apply_rope(k.reshape(1, T, nh, hs), rope).transpose(1, 2)
    v = v.reshape(1, T, nh, hs).transpose(1, 2)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True)  # = the tril mask rows 0..T-1
    x = x + block.attn.c_proj(y.transpose(1, 2).contiguous().view(1, T, C))
    h2 = block.rms_2(x)
    return x + block.mlp.c_proj(F.silu(block.mlp.c_fc1(h2)) * block.mlp.c_fc2(h2))


@torch.no_grad()
def llama_blockwise_quantization(model, sample_inputs, working_device, *, bits=4, groupsize=-1):
    """reference quantize/gptq.py:36-148 (same arguments; `model` holds bf16 nn.Linear layers on
    the GPU, `sample_inputs` (n, T) token ids). Replaces every block Linear and lm_head by a
    ColBlockQuantizedLinear in place; returns the per-Linear quantization errors."""
    dev = torch.device(working_device)
    sample_inputs = sample_inputs.to(dev)
    inps = model.transformer.wte(sample_inputs)
    rope = model.build_rope_cache(sample_inputs)
    outs = torch.zeros_like(inps)
    n = inps.size(0)
    errors = {}
    for i, block in enumerate(model.transformer.h):
        for name in SUBMODULES:
            module = block.get_submodule(name)
            gq = GPTQQuantizer(module, bits=bits, groupsize=groupsize, actorder=(groupsize == -1))
            handle = module.register_forward_hook(gq.collect_input_stats)
            for j in range(n):
                outs[j:j + 1] = calib_block(block, inps[j:j + 1], rope)
            handle.remove()
            q_module, errors[f"transformer.h.{i}.{name}"] = gq.quantize()
            pname, dname = name.rsplit(".", 1)
            setattr(block.get_submodule(pname), dname, q_module)
            del gq
        for j in range(n):
            outs[j:j + 1] = calib_block(block, inps[j:j + 1], rope)
        inps, outs = outs, inps
    for j in range(n):
        outs[j:j + 1] = model.transformer.ln_f(inps[j:j + 1])
    inps, outs = outs, inps
    gq = GPTQQuantizer(model.lm_head, bits=bits, groupsize=groupsize, actorder=(groupsize == -1))
    handle = model.lm_head.register_forward_hook(gq.collect_input_stats)
    for j in range(n):
        model.lm_head(inps[j:j + 1])
    handle.remove()
    model.lm_head, errors["lm_head"] = gq.quantize()
    return errors
