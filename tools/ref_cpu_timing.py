"""Time the REFERENCE's own generate() on the CPU of the build container (SURVEY §8d "CPU
baseline (reference)"), 8 threads, and write profiles/r02_ref_cpu.json. Runs only where
/root/reference exists (it imports the reference exactly as tests/golden/make_golden.py does,
with the same placeholder for the absent `lightning` package); nothing here ships or runs on
the GPU box.

  C0  LLaMAConfig(block_size=128, n_layer=2, n_head=4, n_embd=256) fp32, greedy, 16-token
      prompt, 112 new tokens (the full block): the path generate.py:121 selects without CUDA
  7B fp32 (random weights of the exact shapes), 16-token prompt, 4 new tokens: reduced run
  7B gptq.int4 through the reference's ColBlockQuantizedLinear CPU fallback (get_weight +
      F.linear every call, quantization.py:419-421), 16-token prompt, 2 new tokens: reduced run
Per-token decode time = (t(generate, n new) - t(generate, 1 new)) / (n - 1), i.e. prefill out.
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tests" / "golden"))
import make_golden as MG  # noqa: E402  (reference import + lightning placeholder)
import torch  # noqa: E402

torch.set_num_threads(8)
rgen = MG.rgen
LLaMA, LLaMAConfig = MG.LLaMA, MG.LLaMAConfig


def timed(model, prompt, n):
    t0 = time.perf_counter()
    with torch.no_grad():
        rgen.generate(model, prompt, n, temperature=1.0, top_k=1)
    return time.perf_counter() - t0


def per_token(model, prompt, n):
    model.reset_cache() if model.kv_caches else None
    t1 = timed(model, prompt, 1)
    model.reset_cache()
    tn = timed(model, prompt, n)
    model.reset_cache()
    return (tn - t1) / (n - 1), t1, tn


def main():
    out = {"host": "build container", "threads": torch.get_num_threads(), "reference": "/root/reference generate.generate",
           "runs": []}
    g = torch.Generator().manual_seed(0)
    prompt = torch.randint(3, 32000, (16,), generator=g, dtype=torch.int32)
    # C0
    m = LLaMA(LLaMAConfig(block_size=128, n_layer=2, n_head=4, n_embd=256)).eval()
    dt, t1, tn = per_token(m, prompt, 112)
    out["runs"].append({"config": "C0 fp32 (block_size 128, 2 layers, n_embd 256)", "new_tokens": 112,
                        "decode_s_per_token": dt, "tokens_per_s": 1 / dt, "t_generate_1_s": t1, "t_generate_n_s": tn})
    print(out["runs"][-1], flush=True)
    del m
    # 7B fp32
    with torch.device("meta"):
        m = LLaMA(LLaMAConfig.from_name("7B"))
    m = m.to_empty(device="cpu")
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0.0, 0.02)
    m.eval()
    dt, t1, tn = per_token(m, prompt, 4)
    out["runs"].append({"config": "7B fp32 (random weights)", "new_tokens": 4, "decode_s_per_token": dt,
                        "tokens_per_s": 1 / dt, "t_generate_1_s": t1, "t_generate_n_s": tn})
    print(out["runs"][-1], flush=True)
    del m
    # 7B gptq.int4 through the reference's CPU fallback
    from lit_llama.utils import quantization
    with torch.device("meta"):
        with quantization("gptq.int4"):
            m = LLaMA(LLaMAConfig.from_name("7B"))
    m = m.to_empty(device="cpu")
    with torch.no_grad():
        for name, b in m.named_buffers():
            if name.endswith("quant_weight"):
                b.copy_(torch.randint(0, 256, b.shape, dtype=torch.uint8))
            elif name.endswith("scales"):
                b.uniform_(0.5, 1.5).mul_(0.02 / 7)
            elif name.endswith("zeros"):
                b.fill_(8.0)
        for p in m.parameters():
            p.normal_(0.0, 0.02)
    m.eval()
    dt, t1, tn = per_token(m, prompt, 2)
    out["runs"].append({"config": "7B gptq.int4 (reference CPU fallback: get_weight + F.linear per call)",
                        "new_tokens": 2, "decode_s_per_token": dt, "tokens_per_s": 1 / dt, "t_generate_1_s": t1,
                        "t_generate_n_s": tn})
    print(out["runs"][-1], flush=True)
    (REPO / "profiles" / "r02_ref_cpu.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
