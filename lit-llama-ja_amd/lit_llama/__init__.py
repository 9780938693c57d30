"""lit_llama — MI355X (gfx950) quantized LLaMA decode path, drop-in for the names of
if001/lit-llama-ja's `lit_llama` package (lit_llama/__init__.py:1-2)."""
from lit_llama.model import LLaMAConfig, LLaMA, RMSNorm, build_rope_cache, apply_rope
from lit_llama.tokenizer import Tokenizer, HFTokenizer

__all__ = ["LLaMAConfig", "LLaMA", "RMSNorm", "build_rope_cache", "apply_rope", "Tokenizer", "HFTokenizer"]
