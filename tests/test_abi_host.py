"""CPU tests of the drop-in boundary (no GPU needed).

* the C ABI: every entry point include/lit_llama_amd.h declares is exported by the built
  library, and the ctypes table in lit_llama/_hip.py has the same arity and argument kinds;
  the library carries gfx950 code objects;
* the host-side mirror of the reference interface: lit_llama.utils.quantization /
  EmptyInitOnDevice (reference utils.py:105-194), ColBlockQuantizedLinear buffers and
  state-dict contract (quantization.py:338-367), the LLaMA/LLaMAConfig surface
  (model.py:18-60, lit_llama/__init__.py:1-2), the generate.py CLI flags (92-102);
* that the product path fails loudly off-GPU (no CPU fallback).
"""
import ctypes
import re
import subprocess
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parent.parent
HEADER = REPO / "include" / "lit_llama_amd.h"


def _header_decls():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    decls = {}
    for ret, name, args in re.findall(r"\b(int|size_t)\s+(llj_\w+)\s*\(([^)]*)\)\s*;", text, flags=re.S):
        kinds = []
        for a in args.split(","):
            a = " ".join(a.split())
            if "*" in a:
                kinds.append("p")
            elif a.startswith("float"):
                kinds.append("f")
            elif a.startswith("int"):
                kinds.append("i")
            elif a.startswith("unsigned long long") or a.startswith("size_t"):
                kinds.append("u64")  # ctypes: c_size_t is c_ulong is c_ulonglong on LP64
            else:
                raise AssertionError(f"unexpected argument kind {a!r} in {name}")
        decls[name] = (ret, kinds)
    return decls


def _lib_path():
    from lit_llama import _hip

    if not _hip.LIB_PATH.exists():
        from lit_llama import _build

        _build.build()
    return _hip.LIB_PATH


def test_header_declares_the_abi():
    decls = _header_decls()
    assert len(decls) >= 15
    for name in ("llj_w4_repack", "llj_linear", "llj_norm_qkv_rope", "llj_attention", "llj_linear_resid",
                 "llj_norm_swiglu", "llj_norm_linear", "llj_i8_stats", "llj_i8_quant_weight", "llj_embedding",
                 "llj_rmsnorm", "llj_argmax", "llj_i8_ws_bytes"):
        assert name in decls


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib_path())], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = set(_header_decls()) - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"


def test_library_loads_and_binds_without_gpu():
    L = ctypes.CDLL(str(_lib_path()))
    for name in _header_decls():
        assert getattr(L, name) is not None
    # pure host function: workspace size of the int8 statistics
    L.llj_i8_ws_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    L.llj_i8_ws_bytes.restype = ctypes.c_size_t
    assert L.llj_i8_ws_bytes(8, 4096) > 0


def test_host_options_read_once_and_validated():
    """llj_set_option (host only, no GPU): the A/B options are set / restored per process, invalid
    indices or values are refused (-1000) and never change the table; the LLJ_OPT_* enum of the
    header matches lit_llama._hip's constants."""
    from lit_llama import _hip

    L = ctypes.CDLL(str(_lib_path()))
    text = HEADER.read_text()
    for name, val in re.findall(r"LLJ_OPT_(\w+) = (\d+)", text):
        if name != "COUNT":
            assert getattr(_hip, "OPT_" + name) == int(val), name
    old = L.llj_set_option(_hip.OPT_FLASH_QB, 1)
    assert old in (-1, 1, 2)
    assert L.llj_set_option(_hip.OPT_FLASH_QB, 2) == 1
    assert L.llj_set_option(_hip.OPT_FLASH_QB, 3) == -1000  # out of range: refused, unchanged
    assert L.llj_set_option(_hip.OPT_FLASH_QB, old) == 2
    assert L.llj_set_option(99, 0) == -1000
    assert L.llj_set_option(_hip.OPT_GEMV_LDS_A_KB, 40) == -1000  # below the fused-norm floor (56 KiB)


def test_ctypes_table_matches_header():
    from lit_llama import _hip

    kind = {ctypes.c_void_p: "p", ctypes.c_int: "i", ctypes.c_float: "f", ctypes.c_ulonglong: "u64"}
    decls = _header_decls()
    for name, argt in _hip.SIGNATURES.items():
        assert name in decls, name
        ret, kinds = decls[name]
        assert ret == "int"
        assert [kind[a] for a in argt] == kinds, name
    assert set(decls) - set(_hip.SIGNATURES) == {"llj_i8_ws_bytes", "llj_attention_ws_bytes",
                                                   "llj_g_i8_ws_bytes", "llj_i8_rowstats_bytes",
                                                   "llj_gemm_resid_ws_bytes", "llj_gemm_swiglu_ws_bytes"}


def test_library_holds_gfx950_code():
    data = _lib_path().read_bytes()
    assert b"gfx950" in data


def test_quantization_context_substitutes_and_restores():
    from lit_llama.quantization import ColBlockQuantizedLinear
    from lit_llama.utils import quantization

    orig = torch.nn.Linear
    with quantization("gptq.int4"):
        lin = torch.nn.Linear(256, 64, bias=False)
    assert torch.nn.Linear is orig
    assert isinstance(lin, ColBlockQuantizedLinear) and lin.bits == 4 and lin.tile_cols == 256
    with pytest.raises(ValueError):
        with quantization("nf4"):
            pass
    with pytest.raises(KeyError):
        with quantization("gptq.int4"):
            raise KeyError("body raised")
    assert torch.nn.Linear is orig  # restored even when the body raises
    with quantization(None):
        assert torch.nn.Linear is orig


def test_empty_init_on_device_modes():
    from lit_llama.utils import EmptyInitOnDevice

    with pytest.raises(ValueError):  # reference utils.py:124-126: int8 needs the GPU
        EmptyInitOnDevice(device="cpu", quantization_mode="llm.int8")
    with pytest.raises(RuntimeError):
        EmptyInitOnDevice(device="cpu", quantization_mode="fp3")
    with EmptyInitOnDevice(device="cpu", dtype=torch.bfloat16):
        lin = torch.nn.Linear(32, 16, bias=False)
    assert lin.weight.dtype == torch.bfloat16 and lin.weight.device.type == "cpu"


def test_colblock_buffers_and_state_dict_contract(golden):
    """quant_weight is (N, K/2) uint8 with the reference's column-major strides; the keys
    and shapes equal the GPTQ fixture's (produced by the reference quantize/gptq.py)."""
    from lit_llama.quantization import ColBlockQuantizedLinear

    lin = ColBlockQuantizedLinear(256, 768, False, bits=4, tile_cols=-1)
    assert lin.quant_weight.shape == (768, 128) and lin.quant_weight.stride() == (1, 768)
    assert lin.scales.shape == (768, 1) and lin.zeros.shape == (768, 1)
    assert set(lin.state_dict()) == {"quant_weight", "scales", "zeros"}
    g = golden("int4_gptq")
    key = next(k for k in g if k.endswith("h.0.mlp.c_fc1.quant_weight"))
    qw = torch.from_numpy(g[key])
    sc = torch.from_numpy(g[key.replace("quant_weight", "scales")])
    zr = torch.from_numpy(g[key.replace("quant_weight", "zeros")])
    lin.load_state_dict({"quant_weight": qw, "scales": sc, "zeros": zr})
    assert lin.quant_weight.stride() == (1, 768)  # load copies into the column-major buffer
    assert torch.equal(lin.quant_weight, qw)


def test_colblock_pack_get_weight_roundtrip():
    """pack_weight / get_weight (reference quantization.py:374-409) on CPU."""
    from lit_llama.quantization import ColBlockQuantizedLinear

    torch.manual_seed(0)
    lin = ColBlockQuantizedLinear(64, 32, False, bits=4, tile_cols=-1)
    # power-of-two scales: pack_weight truncates (.to(uint8)) exactly like the reference
    lin.scales.copy_(2.0 ** torch.randint(-6, 0, (32, 1)).float())
    lin.zeros.copy_(torch.randint(0, 16, (32, 1)).float())
    q = torch.randint(0, 16, (32, 64)).float()
    w = (q - lin.zeros) * lin.scales
    lin.pack_weight(w)
    assert torch.equal(lin.quant_weight[:, 0] & 0xF, q[:, 0].to(torch.uint8))  # even k in the low nibble
    assert torch.allclose(lin.get_weight(), w, atol=1e-5)


def test_product_path_has_no_cpu_fallback():
    from lit_llama import _hip
    from lit_llama.quantization import ColBlockQuantizedLinear

    lin = ColBlockQuantizedLinear(128, 32, False, bits=4, tile_cols=-1)
    with pytest.raises(_hip.HipError):
        lin(torch.zeros(1, 128, dtype=torch.bfloat16))
    from lit_llama import LLaMA, LLaMAConfig

    m = LLaMA(LLaMAConfig(block_size=16, vocab_size=512, padded_vocab_size=512, n_layer=1, n_head=2, n_embd=64))
    with pytest.raises(_hip.HipError):
        m(torch.zeros(1, 4, dtype=torch.int32))


def test_unsupported_configs_are_named():
    """Configurations the streaming kernels do not tile are reported with the reason (LLaMAConfig.
    kernel_support); those models run on the any-shape kernels (tests/test_generic_gpu.py)."""
    from lit_llama import LLaMAConfig

    assert "780" in LLaMAConfig.from_name("125M").kernel_support()  # JA fork config, reference model.py:48-51
    assert "not a multiple of 128" in LLaMAConfig(n_layer=16, n_head=16, n_embd=32).kernel_support()
    for name in ("19M", "49M", "7B", "13B", "30B", "65B"):
        assert LLaMAConfig.from_name(name).kernel_support() is None, name


def test_model_api_surface():
    import lit_llama
    from lit_llama import LLaMA, LLaMAConfig
    from lit_llama.utils import find_multiple, llama_model_lookup

    for n in ("LLaMAConfig", "LLaMA", "RMSNorm", "build_rope_cache", "apply_rope", "Tokenizer", "HFTokenizer"):
        assert hasattr(lit_llama, n), n
    c = LLaMAConfig.from_name("7B")
    assert (c.n_layer, c.n_head, c.n_embd, c.block_size, c.padded_vocab_size) == (32, 32, 4096, 2048, 32000)
    assert LLaMAConfig.from_name("13B").n_embd == 5120
    assert find_multiple(int(8 * 4096 / 3), 256) == 11008
    with torch.device("meta"):
        m = LLaMA.from_name("7B")
    assert m.transformer.h[0].mlp.c_fc1.weight.shape == (11008, 4096)
    assert llama_model_lookup({"transformer.wte.weight": torch.empty(1, 5120, device="meta")}) == "13B"


def test_generate_cli_flags():
    out = subprocess.run([sys.executable, str(REPO / "lit-llama-ja_amd" / "generate.py"), "--help"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    for flag in ("--prompt", "--num_samples", "--max_new_tokens", "--top_k", "--temperature", "--checkpoint_path",
                 "--tokenizer_path", "--quantize"):
        assert flag in out.stdout


def test_gptq_cli_flags():
    """quantize/gptq.py keeps the reference CLI (quantize/gptq.py:150-158) plus the offline
    calibration source."""
    out = subprocess.run([sys.executable, str(REPO / "lit-llama-ja_amd" / "quantize" / "gptq.py"), "--help"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    for flag in ("--checkpoint_path", "--output_path", "--tokenizer_path", "--n_samples", "--dtype", "--quantize",
                 "--calibration_path", "--block_size"):
        assert flag in out.stdout


def test_gptq_cli_tokenizer_selection(tmp_path):
    """quantize/gptq.py takes the reference's SentencePiece Tokenizer for its default
    `tokenizer.model` path (reference quantize/gptq.py:17, 207) and the HF JSON tokenizer for a
    `.json` file; a SentencePiece model trained here encodes with BOS like the reference's."""
    sentencepiece = pytest.importorskip("sentencepiece")
    from lit_llama import HFTokenizer, Tokenizer
    from quantize.gptq import tokenizer_for

    corpus = tmp_path / "c.txt"
    corpus.write_text("\n".join(f"the quick brown fox {i} jumps over the lazy dog" for i in range(200)))
    Tokenizer.train(str(corpus), str(tmp_path), vocab_size=60)
    tok = tokenizer_for(tmp_path / "tokenizer.model")
    assert isinstance(tok, Tokenizer)
    ids = tok.encode("the quick brown fox", bos=True)
    assert int(ids[0]) == tok.bos_id and len(ids) > 2
    assert tok.decode(ids[1:]) == "the quick brown fox"
    from tokenizers import Tokenizer as HFTok
    from tokenizers.models import WordLevel

    HFTok(WordLevel({"<pad>": 0, "a": 1}, unk_token="<pad>")).save(str(tmp_path / "t.json"))
    assert isinstance(tokenizer_for(tmp_path / "t.json"), HFTokenizer)
