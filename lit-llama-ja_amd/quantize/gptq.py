"""Whole-model GPTQ driver (reference quantize/gptq.py:36-148, `llama_blockwise_quantization`):
blocks in order, each Linear quantized from the inputs it sees with its predecessors already
quantized, then ln_f and lm_head. The quantizer is lit_llama.quantization.GPTQQuantizer (HIP
column loop + device GEMM / Cholesky). The calibration forward of a block (`calib_block`) runs in
the model's dtype, as the reference does:
  * float32 (the reference CLI's default, quantize/gptq.py:190-203): the reference's own module
    math on the device -- RMSNorm (model.py:276-283), F.linear over fp32 weights (a quantized
    predecessor as F.linear over get_weight(float32), the reference's non-Triton forward,
    quantization.py:419-421), scaled_dot_product_attention with the causal mask;
  * bfloat16: the decode path's kernels (llj_rmsnorm, the HIP ColBlockQuantizedLinear) and torch
    SDPA for the T x T window (opt-in: faster, codes ~60-86 % equal to an fp32 calibration).
The Linears are always called through their modules, so the GPTQ forward hooks fire."""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path
from typing import Optional

if __name__ == "__main__":
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch
import torch.nn.functional as F

from lit_llama.checkpoint import read_checkpoint
from lit_llama.model import apply_rope
from lit_llama.quantization import GPTQQuantizer

SUBMODULES = ["attn.c_attn", "attn.c_proj", "mlp.c_fc1", "mlp.c_fc2", "mlp.c_proj"]  # reference 63-69


def _rmsnorm_ref(norm, x):
    """reference model.py:276-283 in x's dtype (fp32 calibration)."""
    norm_x = torch.mean(x * x, dim=-1, keepdim=True)
    return norm.scale * (x * torch.rsqrt(norm_x + norm.eps))


def _lin(module, x):
    """A Linear of the calibration forward: the module itself (nn.Linear: its GPTQ hook fires), or
    for an already-quantized predecessor in fp32 the reference's non-Triton ColBlock forward."""
    from lit_llama.quantization import ColBlockQuantizedLinear

    if isinstance(module, ColBlockQuantizedLinear) and x.dtype == torch.float32:
        return F.linear(x, module.get_weight(torch.float32), module.bias)
    return module(x)


def calib_block(block, x: torch.Tensor, rope: torch.Tensor) -> torch.Tensor:
    """Block.forward without a KV cache (reference model.py:162-175, 192-242) for one window
    x (1, T, C) in the model's dtype, calling every Linear through its module."""
    _, T, C = x.shape
    nh = block.attn.n_head
    hs = C // nh
    fp32 = x.dtype == torch.float32
    h = _rmsnorm_ref(block.rms_1, x) if fp32 else block.rms_1(x)
    q, k, v = _lin(block.attn.c_attn, h).split(C, dim=2)
    q = apply_rope(q.reshape(1, T, nh, hs), rope).transpose(1, 2)
    k = apply_rope(k.reshape(1, T, nh, hs), rope).transpose(1, 2)
    v = v.reshape(1, T, nh, hs).transpose(1, 2)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True)  # = the tril mask rows 0..T-1
    x = x + _lin(block.attn.c_proj, y.transpose(1, 2).contiguous().view(1, T, C))
    h2 = _rmsnorm_ref(block.rms_2, x) if fp32 else block.rms_2(x)
    return x + _lin(block.mlp.c_proj, F.silu(_lin(block.mlp.c_fc1, h2)) * _lin(block.mlp.c_fc2, h2))


@torch.no_grad()
def llama_blockwise_quantization(model, sample_inputs, working_device, *, bits=4, groupsize=-1):
    """reference quantize/gptq.py:36-148 (same arguments; `model` holds fp32 or bf16 nn.Linear
    layers on the GPU, `sample_inputs` (n, T) token ids). Replaces every block Linear and lm_head by
    a ColBlockQuantizedLinear in place; returns the per-Linear quantization errors."""
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
        x = inps[j:j + 1]
        outs[j:j + 1] = _rmsnorm_ref(model.transformer.ln_f, x) if x.dtype == torch.float32 else model.transformer.ln_f(x)
    inps, outs = outs, inps
    gq = GPTQQuantizer(model.lm_head, bits=bits, groupsize=groupsize, actorder=(groupsize == -1))
    handle = model.lm_head.register_forward_hook(gq.collect_input_stats)
    for j in range(n):
        model.lm_head(inps[j:j + 1])
    handle.remove()
    model.lm_head, errors["lm_head"] = gq.quantize()
    return errors


def tokenizer_for(path: Path):
    """The reference CLI's SentencePiece Tokenizer (quantize/gptq.py:17, 207) for a `.model` file,
    the HF `tokenizers` JSON (HFTokenizer, what the JA fork's generate.py uses) otherwise."""
    from lit_llama import HFTokenizer, Tokenizer

    return Tokenizer(path) if Path(path).suffix == ".model" else HFTokenizer(path)


def get_sample_data(calibration_path=None) -> str:
    """reference quantize/gptq.py:22-33. The reference downloads 1,000 random C4 documents; this
    box has no network, so `calibration_path` (a UTF-8 text file) is the normal source and the
    download is only attempted (as the reference does) when it is not given."""
    if calibration_path is not None:
        return Path(calibration_path).read_text(encoding="utf-8")
    from datasets import load_dataset

    traindata = load_dataset("allenai/c4", "allenai--c4",
                             data_files={"train": "en/c4-train.00000-of-01024.json.gz"}, split="train")
    return "\n".join(traindata[i]["text"] for i in torch.randperm(len(traindata))[:1000].tolist())


def main(*, checkpoint_path: Path = Path("checkpoints/lit-llama/7B/lit-llama.pth"), output_path: Optional[Path] = None,
         tokenizer_path: Path = Path("checkpoints/lit-llama/tokenizer.model"), n_samples: int = 128,
         dtype: str = "float32", quantize: Optional[str] = None, calibration_path: Optional[Path] = None,
         block_size: int = 2048) -> dict:
    """reference quantize/gptq.py:150-237 (same arguments and checks; writes the quantized state
    dict that generate.py --quantize gptq.int4 loads). Differences: the whole model is loaded onto
    the GPU in `dtype` (7B fp32 is 27 GB of 288 GB HBM, so the reference's block-by-block CPU->GPU
    shuttling buys nothing); the calibration text comes from `calibration_path` (no network);
    `block_size` (the reference's fixed 2048) is an argument so small models can be calibrated;
    the tokenizer is the reference's SentencePiece `Tokenizer` for a `.model` file (its default
    path) and the HF `tokenizers` JSON for a `.json` file. Returns the per-Linear errors."""
    from lit_llama import LLaMA
    from lit_llama.utils import EmptyInitOnDevice, llama_model_lookup

    assert checkpoint_path.is_file(), checkpoint_path
    assert tokenizer_path.is_file(), tokenizer_path
    if output_path is None:
        output_path = checkpoint_path.parent / "llama-gptq.4bit.pth"
    assert output_path.parent.is_dir() and (not output_path.exists() or output_path.is_file())
    if not torch.cuda.is_available():
        raise SystemExit("quantize/gptq.py runs on a ROCm GPU (MI355X) only")
    dt = getattr(torch, dtype, None)
    if not isinstance(dt, torch.dtype):
        raise ValueError(f"{dtype} is not a valid dtype.")
    if dt not in (torch.float32, torch.bfloat16):
        raise NotImplementedError(f"calibration in {dtype}: float32 (the reference default) or bfloat16")
    if quantize == "gptq.int4":
        bits = 4
    elif quantize == "gptq.int8":
        bits = 8
    else:
        raise RuntimeError(f"unknown/unsupported quantization mode {quantize}")

    print("Loading model ...", file=sys.stderr)
    t0 = time.time()
    checkpoint = read_checkpoint(checkpoint_path)  # weights only, memory-mapped (incremental_save files too)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=dt):
        model = LLaMA.from_name(llama_model_lookup(checkpoint))
    model.load_state_dict(checkpoint)
    del checkpoint
    print(f"Time to load model: {time.time() - t0:.02f} seconds.", file=sys.stderr)
    model.eval()

    tokenizer = tokenizer_for(tokenizer_path)
    encoded_text = tokenizer.encode(get_sample_data(calibration_path), bos=True, eos=False)
    encoded_text = encoded_text[: n_samples * block_size].reshape(n_samples, block_size)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    errors = llama_blockwise_quantization(model, encoded_text, "cuda", bits=bits)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"\n\nTime for quantization: {t:.02f} sec total", file=sys.stderr)
    print(f"Memory used: {torch.cuda.max_memory_reserved() / 1e9:.02f} GB", file=sys.stderr)
    torch.save(model.state_dict(), output_path)
    return errors


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="GPTQ-quantize a lit-llama checkpoint (reference quantize/gptq.py).")
    ap.add_argument("--checkpoint_path", type=Path, default=Path("checkpoints/lit-llama/7B/lit-llama.pth"))
    ap.add_argument("--output_path", type=Path, default=None)
    ap.add_argument("--tokenizer_path", type=Path, default=Path("checkpoints/lit-llama/tokenizer.model"))
    ap.add_argument("--n_samples", type=int, default=128)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--quantize", default=None, choices=["gptq.int4", "gptq.int8"])
    ap.add_argument("--calibration_path", type=Path, default=None)
    ap.add_argument("--block_size", type=int, default=2048)
    a = ap.parse_args()
    main(checkpoint_path=a.checkpoint_path, output_path=a.output_path, tokenizer_path=a.tokenizer_path,
         n_samples=a.n_samples, dtype=a.dtype, quantize=a.quantize, calibration_path=a.calibration_path,
         block_size=a.block_size)
