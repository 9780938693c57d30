"""HF -> lit-llama checkpoint conversion (reference
scripts/convert_hf_checkpoint.py:19-138) against the reference's own conversion of a tiny
synthetic two-shard HF checkpoint (tests/golden/hf_convert.npz, make_golden.py gen_hf_convert)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest
import torch

from lit_llama import convert as CV
from lit_llama import model as M
from oracle import llama_np as O

GOLD = np.load(Path(__file__).parent / "golden" / "hf_convert.npz")
HF = {k[3:]: torch.from_numpy(GOLD[k]) for k in GOLD.files if k.startswith("hf/")}
LIT = {k[4:]: GOLD[k] for k in GOLD.files if k.startswith("lit/")}
TINY = dict(n_layer=2, n_head=4, n_embd=64, vocab_size=128)


@pytest.fixture
def tiny_config(monkeypatch):
    monkeypatch.setitem(M.llama_configs, "tinyhf", TINY)
    return M.LLaMAConfig.from_name("tinyhf")


def test_state_dict_conversion_matches_reference(tiny_config):
    out = CV.convert_hf_state_dict(HF, tiny_config)
    assert set(out) == set(LIT)
    for k, v in out.items():
        np.testing.assert_array_equal(v.numpy(), LIT[k], err_msg=k)


def test_file_conversion_matches_reference(tiny_config, tmp_path):
    ck = tmp_path / "hf" / "tinyhf"
    ck.mkdir(parents=True)
    (ck / "tokenizer.model").write_bytes(b"placeholder")
    s1 = set(GOLD["shard1_keys"].tolist())
    shards = {"pytorch_model-00001-of-00002.bin": {k: v for k, v in HF.items() if k in s1},
              "pytorch_model-00002-of-00002.bin": {k: v for k, v in HF.items() if k not in s1}}
    for fn, sd in shards.items():
        torch.save(sd, ck / fn)
    wm = {k: fn for fn, sd in shards.items() for k in sd}
    (ck / "pytorch_model.bin.index.json").write_text(json.dumps({"metadata": {}, "weight_map": wm}))
    out = tmp_path / "lit" / "tinyhf"
    CV.convert_hf_checkpoint(output_dir=out, checkpoint_dir=ck, model_size="tinyhf", dtype="float32")
    assert (out.parent / "tokenizer.model").exists()
    sd = torch.load(out / "lit-llama.pth", map_location="cpu", weights_only=True)
    assert set(sd) == set(LIT)
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), LIT[k], err_msg=k)
    # the converted tensors were written straight into the output zip: it is the only file written
    assert sorted(p.name for p in out.iterdir()) == ["lit-llama.pth"]
    with pytest.raises(ValueError):
        CV.convert_hf_checkpoint(output_dir=out, checkpoint_dir=ck, model_size="tinyhf", dtype="float33")


def test_partial_qkv_is_an_error(tiny_config):
    hf = {k: v for k, v in HF.items() if k != "model.layers.1.self_attn.v_proj.weight"}
    with pytest.raises(AssertionError, match="partial"):
        CV.convert_hf_state_dict(hf, tiny_config)


def test_unpermuted_rows_turn_hf_rotary_into_interleaved_rope():
    """Why the permutation: HF's half-split rotary on q = W x equals, after unpermute_rotary on
    the rows, the reference's interleaved apply_rope (model.py:312-329) on the converted rows."""
    n_head, C, T = 4, 64, 5
    hs = C // n_head
    rng = np.random.default_rng(0)
    W = rng.standard_normal((C, C)).astype(np.float32)
    x = rng.standard_normal((T, C)).astype(np.float32)
    q = (x @ W.T).reshape(T, n_head, hs)
    theta = 1.0 / (10000 ** (np.arange(0, hs, 2, dtype=np.float32) / hs))
    ang = np.arange(T, dtype=np.float32)[:, None] * theta[None, :]  # (T, hs/2)
    cos, sin = np.cos(ang)[:, None, :], np.sin(ang)[:, None, :]
    a, b = q[..., :hs // 2], q[..., hs // 2:]
    hf_rot = np.concatenate([a * cos - b * sin, b * cos + a * sin], -1)  # rotate_half form
    Wl = CV.unpermute_rotary(torch.from_numpy(W), n_head).numpy()
    ql = (x @ Wl.T).reshape(1, T, n_head, hs)
    rope = O.build_rope_cache(T, hs)
    lit_rot = O.apply_rope(ql, rope)[0]
    perm = np.stack([np.arange(hs // 2), np.arange(hs // 2) + hs // 2], 1).reshape(-1)  # lit row 2r / 2r+1
    np.testing.assert_allclose(lit_rot, hf_rot[..., perm], rtol=1e-4, atol=1e-4)


def test_load_lit_checkpoint_into_model(tiny_config, tmp_path):
    torch.save({k: torch.from_numpy(v) for k, v in LIT.items()}, tmp_path / "lit-llama.pth")
    tiny_config.block_size = 32
    model = M.LLaMA(tiny_config)
    CV.load_lit_checkpoint(model, tmp_path / "lit-llama.pth")
    np.testing.assert_array_equal(model.transformer.h[1].attn.c_attn.weight.detach().numpy(),
                                  LIT["transformer.h.1.attn.c_attn.weight"])


# ------------------------------------------------------------------ Meta consolidated.*.pth
MGOLD = np.load(Path(__file__).parent / "golden" / "meta_convert.npz")
MPARTS = [{k.split("/", 1)[1]: torch.from_numpy(MGOLD[k]) for k in MGOLD.files if k.startswith(f"meta{r}/")}
          for r in range(2)]
MLIT = {k[4:]: MGOLD[k] for k in MGOLD.files if k.startswith("lit/")}


def test_meta_conversion_matches_reference(tmp_path):
    """Two model-parallel parts merged (sharded dims, c_attn regrouped to Q.. K.. V..) as the
    reference's meta_weights_for_nano_model (convert_checkpoint.py:67-134)."""
    ck = tmp_path / "llama" / "tinymeta"
    ck.mkdir(parents=True)
    (ck.parent / "tokenizer.model").write_bytes(b"placeholder")
    for r, sd in enumerate(MPARTS):
        torch.save(sd, ck / f"consolidated.{r:02d}.pth")
    CV.meta_weights_for_nano_model(output_dir=tmp_path / "lit", checkpoint_dir=tmp_path / "llama",
                                   model_size="tinymeta")
    sd = torch.load(tmp_path / "lit" / "tinymeta" / "lit-llama.pth", map_location="cpu", weights_only=True)
    assert set(sd) == set(MLIT)
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), MLIT[k], err_msg=k)
    with pytest.raises(RuntimeError, match="No checkpoints"):
        CV.meta_weights_for_nano_model(output_dir=tmp_path / "lit", checkpoint_dir=tmp_path / "llama",
                                       model_size="missing")


# ------------------------------------------------------------------ checkpoints the reference wrote
REF_PTH = Path(__file__).parent / "golden" / "ref_lit_llama_bf16.pth"
REF_SUM = np.load(Path(__file__).parent / "golden" / "ref_ckpt.npz")


def _sha(t: torch.Tensor) -> str:
    import hashlib

    return hashlib.sha256(t.contiguous().view(torch.int16).numpy().tobytes()).hexdigest()


def test_reference_incremental_save_file_reads_bitwise():
    """A lit-llama.pth written by the reference's own converter (scripts/convert_hf_checkpoint.py:88
    through its incremental_save, pickle protocol 5; tests/golden/make_golden.py gen_ref_ckpt) reads
    through lazy_load / read_checkpoint with every tensor bit-identical to what the reference's
    lazy_load returned (sha256 per tensor), while torch.load(weights_only=True) refuses it."""
    from lit_llama.checkpoint import read_checkpoint
    from lit_llama.utils import lazy_load

    names = {k[4:] for k in REF_SUM.files if k.startswith("sha/")}
    with lazy_load(REF_PTH) as sd:
        assert set(sd) == names
        for k, v in sd.items():
            assert v.dtype == torch.bfloat16 and str(REF_SUM["dtype/" + k]) == "torch.bfloat16", k
            assert tuple(v.shape) == tuple(REF_SUM["shape/" + k]), k
            assert _sha(v) == str(REF_SUM["sha/" + k]), k
    sd2 = read_checkpoint(REF_PTH)
    assert torch.equal(sd2["lm_head.weight"].view(torch.int16), sd["lm_head.weight"].view(torch.int16))
    import pickle

    with pytest.raises(pickle.UnpicklingError):
        torch.load(REF_PTH, weights_only=True)


def test_lazy_load_refuses_code_in_a_checkpoint(tmp_path):
    """A checkpoint whose pickle names anything but tensors, storages and OrderedDict is refused
    before anything from it runs."""
    import os
    import pickle

    from lit_llama.checkpoint import read_checkpoint

    class Evil:
        def __reduce__(self):
            return (os.system, ("touch " + str(tmp_path / "pwned"),))

    p = tmp_path / "evil.pth"
    w = torch._C.PyTorchFileWriter(str(p))
    data = pickle.dumps({"x": Evil()}, protocol=2)
    w.write_record("data.pkl", data, len(data))
    w.write_end_of_file()
    with pytest.raises(pickle.UnpicklingError, match="posix.system|os.system|refused"):
        read_checkpoint(p)
    assert not (tmp_path / "pwned").exists()


def test_incremental_save_roundtrip(tmp_path):
    """incremental_save (the converters' writer): every dtype / a strided view / an empty tensor,
    written one by one, read back equal by read_checkpoint and by torch.load(weights_only=True)."""
    from lit_llama.checkpoint import incremental_save, read_checkpoint

    base = torch.randn(8, 6)
    tensors = {"f32": torch.randn(3, 5), "bf16": torch.randn(4, 4).to(torch.bfloat16),
               "fp16": torch.randn(7).half(), "u8": torch.randint(0, 255, (5, 3), dtype=torch.uint8),
               "i64": torch.arange(9), "view": base[2:6, 1:4], "empty": torch.empty(0, 3)}
    with incremental_save(tmp_path / "o.pth") as saver:
        saver.save({k: saver.store_early(v) for k, v in tensors.items()})
    for sd in (read_checkpoint(tmp_path / "o.pth"), torch.load(tmp_path / "o.pth", weights_only=True)):
        assert set(sd) == set(tensors)
        for k, v in tensors.items():
            assert sd[k].dtype == v.dtype and torch.equal(sd[k], v), k
    with pytest.raises(RuntimeError):
        with incremental_save(tmp_path / "p.pth") as saver:
            saver.save({})
            saver.save({})
