"""Text generation with the MI355X decode path — drop-in for reference generate.py.

`generate()` keeps the reference signature and semantics (generate.py:18-89): 1-D prompt,
`max_seq_length = min(T + max_new_tokens, block_size)` by default, temperature + top-k
sampling, EOS returns idx[:input_pos] (the EOS token itself is NOT included). Every decode
step runs as one captured HIP graph replay: greedy (top_k=1) ends in the argmax kernel, other
top_k / temperatures in the device top-k sampler.

CLI flags follow reference generate.py:92-102 (argparse; jsonargparse is not installed).
The default CLI decode (top_k=200, temperature=0.8) runs the same captured graph as greedy, with
the device sampler (llj_sample) in place of the argmax.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path
from typing import Optional

import torch

wd = Path(__file__).resolve().parent
sys.path.insert(0, str(wd))

from lit_llama import LLaMA, HFTokenizer  # noqa: E402
from lit_llama.checkpoint import read_checkpoint  # noqa: E402
from lit_llama.engine import DecodeSession  # noqa: E402
from lit_llama.utils import EmptyInitOnDevice, llama_model_lookup  # noqa: E402

EOS_CHECK_EVERY = 16  # greedy graph path: host looks at the ids once per 16 tokens


@torch.no_grad()
def generate(model: LLaMA, idx: torch.Tensor, max_new_tokens: int, *, max_seq_length: Optional[int] = None,
             temperature: float = 1.0, top_k: Optional[int] = None, eos_id: Optional[int] = None) -> torch.Tensor:
    """Takes a conditioning sequence (prompt) as input and continues to generate as many tokens as requested.

    Reference generate.py:18-89. Every decode step, greedy (top_k=1) or sampled, is one replay of
    the captured HIP graph; sampling draws its uniforms from a counter hash seeded from torch's
    default generator, so torch.manual_seed makes a run reproducible as in the reference."""
    T = idx.size(0)
    T_new = T + max_new_tokens
    if max_seq_length is None:
        max_seq_length = min(T_new, model.config.block_size)
    if max_new_tokens <= 0:
        return idx.clone()
    seed = 0 if top_k == 1 else int(torch.randint(0, 2 ** 62, (1,)))
    sess = DecodeSession(model, 1, max_seq_length, T_new, temperature=temperature, top_k=top_k, seed=seed)
    return _run_session(sess, idx, max_new_tokens, eos_id)


def _run_session(sess, idx, max_new_tokens, eos_id):
    T = idx.size(0)
    sess.prefill(idx.view(1, -1))
    left = max_new_tokens - 1
    while True:
        if eos_id is not None:
            gen = sess.output()[0, T:]
            hit = (gen == eos_id).nonzero()
            if hit.numel():  # the reference returns idx[:input_pos]: the EOS token is excluded
                return sess.output()[0, :T + int(hit[0, 0])].to(idx.dtype)
        if left == 0:
            break
        n = min(left, EOS_CHECK_EVERY) if eos_id is not None else left
        sess.decode(n)
        left -= n
    return sess.output()[0].to(idx.dtype)


@torch.no_grad()
def generate_batch(model: LLaMA, idx: torch.Tensor, max_new_tokens: int, *, max_seq_length: Optional[int] = None,
                   eos_id: Optional[int] = None):
    """Greedy decoding of B equal-length prompts (B, T) together (bs=8 throughput mode).
    Each row equals generate(model, idx[b], ..., top_k=1). Returns (B, T + max_new_tokens),
    or with eos_id a list of per-row tensors cut like the reference's EOS rule."""
    B, T = idx.shape
    T_new = T + max_new_tokens
    if max_seq_length is None:
        max_seq_length = min(T_new, model.config.block_size)
    sess = DecodeSession(model, B, max_seq_length, T_new)
    sess.prefill(idx)
    if max_new_tokens > 1:
        sess.decode(max_new_tokens - 1)
    out = sess.output().to(idx.dtype)
    if eos_id is None:
        return out
    rows = []
    for b in range(B):
        hit = (out[b, T:] == eos_id).nonzero()
        rows.append(out[b, :T + int(hit[0, 0])] if hit.numel() else out[b])
    return rows


def main(prompt: str = "Hello, my name is", *, num_samples: int = 1, max_new_tokens: int = 50, top_k: int = 200,
         temperature: float = 0.8, checkpoint_path: Path = Path("checkpoints/lit-llama/7B/lit-llama.pth"),
         tokenizer_path: Path = Path("checkpoints/lit-llama/tokenizer.model"), quantize: Optional[str] = None) -> None:
    """Generates text samples based on a pre-trained LLaMA model and tokenizer (reference generate.py:92-155)."""
    assert checkpoint_path.is_file(), checkpoint_path
    assert tokenizer_path.is_file(), tokenizer_path
    if not torch.cuda.is_available():
        raise SystemExit("this generate.py runs on a ROCm GPU (MI355X) only")
    print("Loading model ...", file=sys.stderr)
    t0 = time.time()
    checkpoint = read_checkpoint(checkpoint_path)  # weights only, memory-mapped (incremental_save files too)
    name = llama_model_lookup(checkpoint)
    with EmptyInitOnDevice(device=torch.device("cuda"), dtype=torch.bfloat16, quantization_mode=quantize):
        model = LLaMA.from_name(name)
    model.load_state_dict(checkpoint)
    del checkpoint
    print(f"Time to load model: {time.time() - t0:.02f} seconds.", file=sys.stderr)
    model.eval()
    tokenizer = HFTokenizer(tokenizer_path)
    encoded = tokenizer.encode(prompt, bos=True, eos=False, device=torch.device("cuda"))
    prompt_length = encoded.size(0)
    torch.manual_seed(1234)
    for i in range(num_samples):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = generate(model, encoded, max_new_tokens, temperature=temperature, top_k=top_k)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        model.reset_cache()
        print(tokenizer.decode(y))
        tokens_generated = y.size(0) - prompt_length
        print(f"Time for inference {i + 1}: {t:.02f} sec total, {tokens_generated / t:.02f} tokens/sec", file=sys.stderr)
    print(f"Memory used: {torch.cuda.max_memory_reserved() / 1e9:.02f} GB", file=sys.stderr)


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="Generates text samples based on a pre-trained LLaMA model and tokenizer.")
    ap.add_argument("--prompt", default="Hello, my name is")
    ap.add_argument("--num_samples", type=int, default=1)
    ap.add_argument("--max_new_tokens", type=int, default=50)
    ap.add_argument("--top_k", type=int, default=200)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--checkpoint_path", type=Path, default=Path("checkpoints/lit-llama/7B/lit-llama.pth"))
    ap.add_argument("--tokenizer_path", type=Path, default=Path("checkpoints/lit-llama/tokenizer.model"))
    ap.add_argument("--quantize", default=None, choices=[None, "llm.int8", "gptq.int4", "gptq.int8"])
    a = ap.parse_args()
    main(a.prompt, num_samples=a.num_samples, max_new_tokens=a.max_new_tokens, top_k=a.top_k,
         temperature=a.temperature, checkpoint_path=a.checkpoint_path, tokenizer_path=a.tokenizer_path,
         quantize=a.quantize)
