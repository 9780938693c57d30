"""Perplexity of a (quantized) LLaMA over fixed windows -- drop-in for reference evaluate/full.py
(main 46-140, the loop 114-129): the text is encoded with the SentencePiece Tokenizer (BOS, no
EOS), trimmed to 256 * block_size tokens, and cut into windows of 2048 tokens; every window is one
no-cache LLaMA.forward (prompt rows through the MFMA prefill GEMMs and the flash attention) whose
logits[:-1] score inp[1:] with a summed cross entropy. ppl = exp(sum nll / tokens scored).

The reference fetches wikitext / ptb / c4 with `datasets` (evaluate/full.py:23-43); without a
network the text comes from files (`--text_path`, one or more, comma separated)."""
from __future__ import annotations

import argparse
import math
import sys
import time
from pathlib import Path
from typing import Optional

import torch

wd = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(wd))

from lit_llama import LLaMA  # noqa: E402
from lit_llama.checkpoint import read_checkpoint  # noqa: E402
from lit_llama.utils import EmptyInitOnDevice  # noqa: E402

WINDOW = 2048  # reference evaluate/full.py:117 ("for compat with gptq")


@torch.no_grad()
def perplexity(model: LLaMA, encoded_text: torch.Tensor, window: int = WINDOW):
    """reference evaluate/full.py:114-128 over `encoded_text` (1, N) on the model's device:
    returns (ppl, summed nll, tokens scored)."""
    nlls, toks = 0.0, 0
    window = min(window, model.config.block_size)
    for i in range(0, encoded_text.shape[1], window):
        inp = encoded_text[:, i:i + window]
        if inp.shape[1] < 2:
            break
        logits = model(inp)[0]
        nll = torch.nn.functional.cross_entropy(logits[:-1].float(), inp[0, 1:].to(dtype=torch.long), reduction="sum")
        toks += inp.size(1) - 1
        nlls += nll.item()
    return math.exp(nlls / toks), nlls, toks


def main(text_path: str, *, checkpoint_path: Optional[Path] = None,
         tokenizer_path: Path = Path("checkpoints/lit-llama/tokenizer.model"), model_size: str = "7B",
         dtype: str = "float32", quantize: Optional[str] = None) -> dict:
    """reference evaluate/full.py:46-140 (same flags, dtype default float32 as there: an fp32 model
    runs every op on the any-shape kernels in fp32; bfloat16 takes the fused MFMA prefill path)."""
    from quantize.gptq import tokenizer_for

    dt = getattr(torch, dtype, None)
    if not isinstance(dt, torch.dtype):  # reference evaluate/full.py:78-81
        raise ValueError(f"{dtype} is not a valid dtype.")
    if not checkpoint_path:
        checkpoint_path = Path(f"checkpoints/lit-llama/{model_size}/lit-llama.pth")
    assert checkpoint_path.is_file() and tokenizer_path.is_file()
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=dt, quantization_mode=quantize):
        print("Loading model ...", file=sys.stderr)
        t0 = time.time()
        model = LLaMA.from_name(model_size)
        model.load_state_dict(read_checkpoint(checkpoint_path))  # weights only, memory-mapped
        print(f"Time to load model: {time.time() - t0:.02f} seconds.", file=sys.stderr)
    model.eval()
    tokenizer = tokenizer_for(tokenizer_path)
    out, total_toks = {}, 0
    t0 = time.perf_counter()
    for path in text_path.split(","):
        enc = tokenizer.encode(Path(path).read_text(encoding="utf-8"), bos=True, eos=False,
                               device=torch.device("cuda"))[None, :256 * model.config.block_size]
        ppl, _, toks = perplexity(model, enc)
        print(f"Perplexity on {path}: {ppl:.2f}")
        out[path] = ppl
        total_toks += toks
    t = time.perf_counter() - t0
    print(f"\n\nTime for inference: {t:.02f} sec total, {total_toks / t:.02f} tokens/sec", file=sys.stderr)
    print(f"Memory used: {torch.cuda.max_memory_reserved() / 1e9:.02f} GB", file=sys.stderr)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="Perplexity of a lit-llama checkpoint (reference evaluate/full.py).")
    ap.add_argument("--text_path", required=True)
    ap.add_argument("--checkpoint_path", type=Path, default=None)
    ap.add_argument("--tokenizer_path", type=Path, default=Path("checkpoints/lit-llama/tokenizer.model"))
    ap.add_argument("--model_size", default="7B")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--quantize", default=None, choices=[None, "llm.int8", "gptq.int4", "gptq.int8"])
    a = ap.parse_args()
    main(a.text_path, checkpoint_path=a.checkpoint_path, tokenizer_path=a.tokenizer_path, model_size=a.model_size,
         dtype=a.dtype, quantize=a.quantize)
