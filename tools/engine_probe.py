"""Profiling aid for rocprofv3 counter passes over the persistent decode engine (csrc/engine.hip):
LLaMA-7B gptq.int4 bs=1 (bench.py's synthetic model), eager launches of llj_engine_step in a fixed
order so the dispatch rows of a --pmc pass can be told apart:
  dispatches 0..2  consumers alone (every ring block "landed", nothing streamed: flags bit 2)
  dispatches 3..5  the real step (loader + consumers)
  dispatches 6..8  the loader alone (flags bit 1)
Usage: rocprofv3 --pmc <counters> -- python3 tools/engine_probe.py
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))

import bench  # noqa: E402


def main():
    from lit_llama.engine import DecodeSession

    os.environ["LLJ_ENGINE"] = "1"
    model = bench.build_model("7B", "gptq.int4")
    prompt = torch.randint(3, 32000, (1, 16), generator=torch.Generator().manual_seed(1)).cuda()
    s = DecodeSession(model, 1, 144, 16 + 40, use_graph=False)
    s.prefill(prompt)
    assert s.engine is not None, s.engine_off_reason
    s.decode(4)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    print("probe: consumers alone x3", flush=True)
    for _ in range(3):
        s.engine.probe_consumers(st)
    torch.cuda.synchronize()
    s2 = DecodeSession(model, 1, 144, 16 + 40, use_graph=False)  # the consumers-alone launches left state invalid
    s2.prefill(prompt)
    s2.decode(1)
    torch.cuda.synchronize()
    print("probe: real steps x3", flush=True)
    for _ in range(3):
        s2.engine.step(st)
    torch.cuda.synchronize()
    print("probe: loader alone x3", flush=True)
    for _ in range(3):
        s2.engine.probe_stream(st)
    torch.cuda.synchronize()
    print("probe done", flush=True)


if __name__ == "__main__":
    main()
