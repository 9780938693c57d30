"""Checkpoint formats: Hugging Face LLaMA shards -> lit-llama state dict.

Mirrors reference scripts/convert_hf_checkpoint.py:19-138 (`convert_hf_checkpoint`, same keyword
arguments and output file `lit-llama.pth`, tokenizer copied to the output's parent): the HF
per-projection q / k / v weights are fused into `attn.c_attn.weight` with q and k rows permuted
from HF's half-split rotary layout back to the interleaved pairs `apply_rope` uses
(model.py:312-329; the inverse of transformers' convert_llama_weights_to_hf permute), every other
tensor renamed by the reference's weight map, `rotary_emb.inv_freq` dropped. Input shards are read
memory-mapped and weights-only (checkpoint.read_checkpoint: nothing in a checkpoint is executed);
every converted tensor goes straight into the output zip through checkpoint.incremental_save as
soon as it exists (the reference's own scheme, lit_llama/utils.py:492-531), so the process holds at
most one converted tensor in memory and the output is the only file written (about one model size
of disk). `load_lit_checkpoint` streams a lit-llama.pth straight into a model's (device) parameters.
"""
from __future__ import annotations

import json
import shutil
from pathlib import Path

import torch

from .checkpoint import incremental_save, read_checkpoint
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
        hf.update(read_checkpoint(b))
    with incremental_save(output_dir / "lit-llama.pth") as saver:
        saver.save(convert_hf_state_dict(hf, config, dt, saver.store_early))


def load_lit_checkpoint(model: torch.nn.Module, path: Path, strict: bool = True):
    """Load lit-llama.pth into `model` (its parameters may already live on the GPU): the file
    is memory-mapped and each tensor copied into its parameter once (reference lazy_load +
    load_state_dict, utils.py:200-376)."""
    sd = read_checkpoint(Path(path))
    return model.load_state_dict(sd, strict=strict)


# ----------------------------------------------------------------------- Meta (consolidated.*.pth)
# reference scripts/convert_checkpoint.py:20-53: lit-llama name -> Meta name(s) (per layer / global)
_META_TOP = {"transformer.wte.weight": "tok_embeddings.weight", "lm_head.weight": "output.weight",
             "transformer.ln_f.scale": "norm.weight"}
_META_LAYER = {"attn.c_attn.weight": ("attention.wq.weight", "attention.wk.weight", "attention.wv.weight"),
               "attn.c_proj.weight": ("attention.wo.weight",), "mlp.c_fc1.weight": ("feed_forward.w1.weight",),
               "mlp.c_proj.weight": ("feed_forward.w2.weight",), "mlp.c_fc2.weight": ("feed_forward.w3.weight",),
               "rms_1.scale": ("attention_norm.weight",), "rms_2.scale": ("ffn_norm.weight",)}


def meta_names(state_dict: dict) -> list:
    """lit-llama names of a Meta state dict, in the reference converter's order."""
    layers = sorted({k.split(".")[1] for k in state_dict if k.startswith("layers")})
    return list(_META_TOP) + [f"transformer.h.{i}.{n}" for i in layers for n in _META_LAYER]


def meta_tensor(state_dict: dict, name: str, dtype=torch.float32) -> torch.Tensor:
    """One lit-llama tensor from a Meta state dict (wq / wk / wv stacked into c_attn; Meta's rotary
    layout is already the interleaved one)."""
    if name in _META_TOP:
        return state_dict[_META_TOP[name]].to(dtype)
    _, _, i, rest = name.split(".", 3)
    src = [state_dict[f"layers.{i}.{m}"].to(dtype) for m in _META_LAYER[rest]]
    return torch.cat(src) if len(src) > 1 else src[0]


def convert_meta_state_dict(state_dict: dict, dtype=torch.float32, sink=None) -> dict:
    """reference scripts/convert_checkpoint.py:20-53 for one part. `sink` as in
    convert_hf_state_dict."""
    keep = sink if sink is not None else (lambda t: t)
    return {n: keep(meta_tensor(state_dict, n, dtype)) for n in meta_names(state_dict)}


# model-parallel split dimension per tensor (reference convert_checkpoint.py:56-64)
SHARD_DIMS = {"lm_head.weight": 0, "wte.weight": 1, "attn.c_attn.weight": 0, "attn.c_proj.weight": 1,
              "mlp.c_fc1.weight": 0, "mlp.c_fc2.weight": 0, "mlp.c_proj.weight": 1}


def merge_meta_tensor(name: str, parts: list) -> torch.Tensor:
    """One tensor from its model-parallel parts (convert_checkpoint.py:95-113; unsharded tensors
    are taken from the first part), c_attn regrouped from [Q1 K1 V1 Q2 K2 V2 ...] to
    [Q1 Q2 ... K1 K2 ... V1 V2 ...] (115-131)."""
    n = len(parts)
    dim = next((d for k, d in SHARD_DIMS.items() if k in name), None)
    t = torch.cat(parts, dim=dim) if (dim is not None and n > 1) else parts[0]
    if "c_attn" in name:
        src = t.shape[0] // n
        mat = src // 3
        t = torch.cat([t[i * src + j * mat: i * src + (j + 1) * mat] for j in range(3) for i in range(n)])
    return t


def merge_meta_shards(converted: list, sink=None) -> dict:
    """Merge converted parts tensor by tensor (merge_meta_tensor), each merged result handed to
    `sink` (as in convert_hf_state_dict) before the next is built."""
    keep = sink if sink is not None else (lambda t: t)
    return {name: keep(merge_meta_tensor(name, [part[name] for part in converted])) for name in converted[0]}


@torch.no_grad()
def meta_weights_for_nano_model(*, output_dir: Path = Path("checkpoints/lit-llama"),
                                checkpoint_dir: Path = Path("checkpoints/llama/"), model_size: str = "7B",
                                dtype: str = "float32") -> None:
    """reference convert_checkpoint.py:67-134 (same arguments and layout: <dir>/<size>/...). The
    parts are memory-mapped; each output tensor is built from its slices of every part and written
    into the output zip before the next one is built."""
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
    parts = [read_checkpoint(f) for f in files]
    with incremental_save(output_dir / "lit-llama.pth") as saver:
        out = {}
        for name in meta_names(parts[0]):
            out[name] = saver.store_early(merge_meta_tensor(name, [meta_tensor(p, name, dt) for p in parts]))
        saver.save(out)
