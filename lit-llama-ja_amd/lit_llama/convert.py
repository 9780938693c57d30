"""Checkpoint formats: Hugging Face LLaMA shards -> lit-llama state dict.

Mirrors reference scripts/convert_hf_checkpoint.py:19-138 (`convert_hf_checkpoint`, same keyword
arguments and output file `lit-llama.pth`, tokenizer copied to the output's parent): the HF
per-projection q / k / v weights are fused into `attn.c_attn.weight` with q and k rows permuted
from HF's half-split rotary layout back to the interleaved pairs `apply_rope` uses
(model.py:312-329; the inverse of transformers' convert_llama_weights_to_hf permute), every other
tensor renamed by the reference's weight map, `rotary_emb.inv_freq` dropped. Shards are opened
memory-mapped with `torch.load(weights_only=True, mmap=True)` (nothing in a checkpoint is
executed); every converted tensor is spilled into a file-backed (memory-mapped) storage next to
the output as soon as it exists, so the final `torch.save` streams from the page cache and the
process never holds more than one converted tensor in anonymous memory (the reference gets the
same bound from its incremental_save, lit_llama/utils.py). `load_lit_checkpoint` streams a
lit-llama.pth straight into a model's (device) parameters.
"""
from __future__ import annotations

import json
import shutil
import tempfile
from pathlib import Path

import torch

from .model import LLaMAConfig

# reference convert_hf_checkpoint.py:74-87
WEIGHT_MAP = {
    "self_attn.o_proj.weight": "attn.c_proj.weight",
    "self_attn.q_proj.weight": "attn.c_attn.weight",
    "self_attn.k_proj.weight": "attn.c_attn.weight",
    "self_attn.v_proj.weight": "attn.c_attn.weight",
    "mlp.gate_proj.weight": "mlp.c_fc1.weight",
    "mlp.up_proj.weight": "mlp.c_fc2.weight",
    "mlp.down_proj.weight": "mlp.c_proj.weight",
    "input_layernorm.weight": "rms_1.scale",
    "post_attention_layernorm.weight": "rms_2.scale",
    "model.embed_tokens.weight": "transformer.wte.weight",
    "model.norm.weight": "transformer.ln_f.scale",
    "lm_head.weight": "lm_head.weight",
}


def unpermute_rotary(w: torch.Tensor, n_head: int) -> torch.Tensor:
    """HF half-split rotary rows -> interleaved pairs (reference convert_hf_checkpoint.py:63-70):
    within each head, row r of the first half and row r of the second half become rows 2r, 2r+1."""
    dim = w.shape[1]
    return w.view(n_head, 2, dim // n_head // 2, dim).transpose(1, 2).reshape(dim, dim)


class _Spill:
    """Sink for converted tensors: each one is copied into its own memory-mapped file in `dir` and
    the file-backed tensor is kept instead (its pages are the kernel's to write back and drop)."""

    def __init__(self, dir: Path):
        self.dir = Path(tempfile.mkdtemp(prefix=".lit-convert-", dir=dir))
        self.n = 0

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        t = t.contiguous()
        f = self.dir / f"{self.n}.bin"
        self.n += 1
        m = torch.from_file(str(f), shared=True, size=t.numel(), dtype=t.dtype).view(t.shape)
        m.copy_(t)
        return m

    def close(self):
        shutil.rmtree(self.dir, ignore_errors=True)


def _save_spilled(make, out_path: Path) -> None:
    """torch.save of the state dict make(sink) builds, every tensor spilled as it is made."""
    sink = _Spill(out_path.parent)
    try:
        torch.save(make(sink), out_path)
    finally:
        sink.close()


def convert_hf_state_dict(hf: dict, config: LLaMAConfig, dtype=torch.float32, sink=None) -> dict:
    """Map one HF LLaMA state dict (possibly merged from all shards) to lit-llama keys; `sink`
    (optional) receives each converted tensor and returns what the result dict keeps."""
    keep = sink if sink is not None else (lambda t: t)
    out, qkv = {}, {}
    for name, t in hf.items():
        if "rotary_emb.inv_freq" in name:
            continue
        if "model.layers" in name:
            parts = name.split(".")
            key = f"transformer.h.{int(parts[2])}.{WEIGHT_MAP['.'.join(parts[3:])]}"
            proj = parts[4] if parts[3] == "self_attn" and parts[4] in ("q_proj", "k_proj", "v_proj") else None
            if proj is not None:
                qkv.setdefault(key, {})[proj] = t
                if len(qkv[key]) == 3:
                    parts3 = qkv.pop(key)
                    out[key] = keep(torch.cat([unpermute_rotary(parts3["q_proj"].to(dtype), config.n_head),
                                               unpermute_rotary(parts3["k_proj"].to(dtype), config.n_head),
                                               parts3["v_proj"].to(dtype)], 0))
                continue
            out[key] = keep(t.to(dtype))
        else:
            out[WEIGHT_MAP[name]] = keep(t.to(dtype))
    if qkv:  # reference convert_hf_checkpoint.py:137
        raise AssertionError(f"unexpected partial weights {list(qkv)}")
    return out


@torch.no_grad()
def convert_hf_checkpoint(*, output_dir: Path = Path("checkpoints/lit-llama/7B"),
                          checkpoint_dir: Path = Path("checkpoints/hf-llama/7B"), model_size: str = "7B",
                          dtype: str = "float32", verify: bool = False) -> None:
    """File-level converter with the reference's arguments (verify needs transformers' model
    download and is not supported offline)."""
    output_dir, checkpoint_dir = Path(output_dir), Path(checkpoint_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    shutil.copy(checkpoint_dir / "tokenizer.model", output_dir.parent)
    dt = getattr(torch, dtype, None)
    if not isinstance(dt, torch.dtype):
        raise ValueError(f"{dtype} is not a valid dtype.")
    if verify:
        raise NotImplementedError("verify=True compares against transformers' LlamaForCausalLM.from_pretrained")
    config = LLaMAConfig.from_name(model_size)
    with open(checkpoint_dir / "pytorch_model.bin.index.json") as f:
        bin_index = json.load(f)
    bin_files = sorted(set(checkpoint_dir / b for b in bin_index["weight_map"].values()))
    if not bin_files:
        raise ValueError(f"Expected {str(checkpoint_dir)!r} to contain .bin files")
    hf = {}
    for b in bin_files:  # memory-mapped: tensors are read when converted
        hf.update(torch.load(b, map_location="cpu", weights_only=True, mmap=True))
    _save_spilled(lambda sink: convert_hf_state_dict(hf, config, dt, sink), output_dir / "lit-llama.pth")


def load_lit_checkpoint(model: torch.nn.Module, path: Path, strict: bool = True):
    """Load lit-llama.pth into `model` (its parameters may already live on the GPU): the file
    is memory-mapped and each tensor copied into its parameter once (reference lazy_load +
    load_state_dict, utils.py:200-376, without the custom unpickler)."""
    sd = torch.load(Path(path), map_location="cpu", weights_only=True, mmap=True)
    return model.load_state_dict(sd, strict=strict)


# ----------------------------------------------------------------------- Meta (consolidated.*.pth)
def convert_meta_state_dict(state_dict: dict, dtype=torch.float32, sink=None) -> dict:
    """reference scripts/convert_checkpoint.py:20-53: Meta names -> lit-llama names, wq / wk / wv
    stacked into c_attn (Meta's rotary layout is already the interleaved one). `sink` as in
    convert_hf_state_dict."""
    keep = sink if sink is not None else (lambda t: t)
    out = {"transformer.wte.weight": keep(state_dict["tok_embeddings.weight"].to(dtype)),
           "lm_head.weight": keep(state_dict["output.weight"].to(dtype)),
           "transformer.ln_f.scale": keep(state_dict["norm.weight"].to(dtype))}
    layers = sorted({k.split(".")[1] for k in state_dict if k.startswith("layers")})
    for i in layers:
        p, q = f"layers.{i}.", f"transformer.h.{i}."
        out[q + "attn.c_attn.weight"] = keep(torch.cat([state_dict[p + f"attention.{w}.weight"].to(dtype)
                                                        for w in ("wq", "wk", "wv")]))
        out[q + "attn.c_proj.weight"] = keep(state_dict[p + "attention.wo.weight"].to(dtype))
        out[q + "mlp.c_fc1.weight"] = keep(state_dict[p + "feed_forward.w1.weight"].to(dtype))
        out[q + "mlp.c_proj.weight"] = keep(state_dict[p + "feed_forward.w2.weight"].to(dtype))
        out[q + "mlp.c_fc2.weight"] = keep(state_dict[p + "feed_forward.w3.weight"].to(dtype))
        out[q + "rms_1.scale"] = keep(state_dict[p + "attention_norm.weight"].to(dtype))
        out[q + "rms_2.scale"] = keep(state_dict[p + "ffn_norm.weight"].to(dtype))
    return out


# model-parallel split dimension per tensor (reference convert_checkpoint.py:56-64)
SHARD_DIMS = {"lm_head.weight": 0, "wte.weight": 1, "attn.c_attn.weight": 0, "attn.c_proj.weight": 1,
              "mlp.c_fc1.weight": 0, "mlp.c_fc2.weight": 0, "mlp.c_proj.weight": 1}


def merge_meta_shards(converted: list, sink=None) -> dict:
    """Concatenate the model-parallel parts (convert_checkpoint.py:95-113; unsharded tensors are
    taken from the first part) and regroup c_attn from [Q1 K1 V1 Q2 K2 V2 ...] to
    [Q1 Q2 ... K1 K2 ... V1 V2 ...] (115-131). Tensor by tensor, each merged result handed to
    `sink` (as in convert_hf_state_dict) before the next is built."""
    keep = sink if sink is not None else (lambda t: t)
    n = len(converted)
    combined = {}
    for name, t0 in converted[0].items():
        dim = next((d for k, d in SHARD_DIMS.items() if k in name), None)
        t = torch.cat([part[name] for part in converted], dim=dim) if (dim is not None and n > 1) else t0
        if "c_attn" in name:
            src = t.shape[0] // n
            mat = src // 3
            t = torch.cat([t[i * src + j * mat: i * src + (j + 1) * mat] for j in range(3) for i in range(n)])
        combined[name] = keep(t)
        del t
    return combined


@torch.no_grad()
def meta_weights_for_nano_model(*, output_dir: Path = Path("checkpoints/lit-llama"),
                                checkpoint_dir: Path = Path("checkpoints/llama/"), model_size: str = "7B",
                                dtype: str = "float32") -> None:
    """reference convert_checkpoint.py:67-134 (same arguments and layout: <dir>/<size>/...)."""
    output_dir, checkpoint_dir = Path(output_dir) / model_size, Path(checkpoint_dir) / model_size
    output_dir.mkdir(parents=True, exist_ok=True)
    shutil.copy(checkpoint_dir.parent / "tokenizer.model", output_dir.parent)
    dt = getattr(torch, dtype, None)
    if not isinstance(dt, torch.dtype):
        raise ValueError(f"{dtype} is not a valid dtype.")
    files = sorted(checkpoint_dir.glob("*.pth"))
    if not files:
        raise RuntimeError(f"No checkpoints were found at checkpoint_dir {checkpoint_dir}. "
                           "`consolidated.0*.pth` files expected at that location.")
    def make(sink):
        # every part converted into spilled (file-backed) tensors, then merged tensor by tensor
        parts = [convert_meta_state_dict(torch.load(f, map_location="cpu", weights_only=True, mmap=True), dt, sink)
                 for f in files]
        return merge_meta_shards(parts, sink)

    _save_spilled(make, output_dir / "lit-llama.pth")
