"""Profiling aid: per-CU phase stamps of the persistent decode engine (csrc/engine.hip STAMP
indices) for LLaMA-7B gptq.int4 bs=1 (bench.py's synthetic model), and the engine vs launch-chain
step time. Prints the median / max over CUs of each phase's end time relative to the step start.

Usage: python tools/engine_trace.py [--layers 32] [--out gpurun_out/engine_trace.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))

import bench  # noqa: E402

NAMES = ["x staged", "QKV done", "attn done", "y staged", "c_proj done", "x_mid staged", "SwiGLU done", "h staged",
         "down done"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "engine_trace.json"))
    args = ap.parse_args()
    from lit_llama import LLaMA, LLaMAConfig
    from lit_llama.engine import DecodeSession
    from lit_llama.utils import EmptyInitOnDevice

    if args.layers == 32:
        model = bench.build_model("7B", "gptq.int4")
    else:
        dev = torch.device("cuda")
        with EmptyInitOnDevice(device=dev, dtype=torch.bfloat16, quantization_mode="gptq.int4"):
            model = LLaMA(LLaMAConfig(n_layer=args.layers, n_head=32, n_embd=4096))
        g = torch.Generator(device=dev).manual_seed(1)
        with torch.no_grad():
            for mod in model.modules():
                if hasattr(mod, "quant_weight"):
                    mod.quant_weight.copy_(torch.randint(0, 256, mod.quant_weight.shape, device=dev, dtype=torch.uint8,
                                                         generator=g))
                    mod.scales.copy_((torch.rand(mod.scales.shape, device=dev, generator=g) + 0.5) * (0.02 / 7))
                    mod.zeros.fill_(8.0)
                elif isinstance(mod, torch.nn.Embedding):
                    mod.weight.normal_(0.0, 0.02, generator=g)
    prompt = torch.randint(3, 32000, (1, 16), generator=torch.Generator().manual_seed(1)).cuda()
    res = {}
    for eng in (True, False):
        os.environ["LLJ_ENGINE"] = "1" if eng else "0"
        s = DecodeSession(model, 1, 144, 16 + 100)
        s.prefill(prompt)
        assert (s.engine is not None) == eng, s.engine_off_reason
        s.decode(50)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.decode(40)
        e1.record()
        torch.cuda.synchronize()
        res["engine_us" if eng else "chain_us"] = e0.elapsed_time(e1) / 40 * 1e3
        if eng:
            assert s.engine.error_bits() == 0
            tr = s.engine.enable_trace()
            st = torch.cuda.current_stream().cuda_stream
            s.engine.probe_stream(st)  # loader alone: the raw in-engine stream rate
            torch.cuda.synchronize()
            t = tr.view(-1, 128).cpu().numpy().astype(np.float64)
            G = int((t[:, 120] > 0).sum())
            t = t[:G]
            st0 = t[:, 121:122]
            res["probe_loader_op_issued"] = [float(np.median((t[:, 100 + i] - st0[:, 0]) / 100.0)) for i in range(8)]
            res["probe_stream_end_us"] = float(np.median((t[:, 120] - st0[:, 0]) / 100.0))
            # the same probe with every layer's weights copied into ONE allocation (layer-major, op
            # order): does the weights' placement set the stream rate?
            from lit_llama.engine import _EngLayer
            eng_ = s.engine
            n_l = model.config.n_layer
            lay = (_EngLayer * n_l).from_buffer_copy(bytes(eng_.layers.cpu().numpy().tobytes()))
            ws = [eng_.keep[12 * i + k] for i in range(n_l) for k in (0, 2, 4, 6, 8)]
            tot = sum(w.numel() * w.element_size() for w in ws)
            big = torch.empty(tot + 4096 * len(ws), dtype=torch.uint8, device="cuda")
            off, newp = 0, []
            for w in ws:
                nbytes = w.numel() * w.element_size()
                big[off:off + nbytes].copy_(w.reshape(-1).view(torch.uint8))
                newp.append(big.data_ptr() + off)
                off += (nbytes + 4095) // 4096 * 4096
            for i in range(n_l):
                lay[i].w_qkv, lay[i].w_o, lay[i].w_fc1, lay[i].w_fc2, lay[i].w_down = newp[5 * i:5 * i + 5]
            saved_layers = eng_.layers
            eng_.layers = torch.frombuffer(bytearray(bytes(lay)), dtype=torch.uint8).to("cuda")
            eng_.plan.layers = eng_.layers.data_ptr()
            tr.zero_()
            eng_.probe_stream(st)
            torch.cuda.synchronize()
            t = tr.view(-1, 128).cpu().numpy().astype(np.float64)[:G]
            res["probe_one_alloc_stream_end_us"] = float(np.median((t[:, 120] - t[:, 121]) / 100.0))
            eng_.layers = saved_layers
            eng_.plan.layers = eng_.layers.data_ptr()
            del big
            tr.zero_()
            s.graph = None  # recapture with the trace pointer
            s.decode(2)
            torch.cuda.synchronize()
            traced = tr.clone()
            # consumers alone (nothing streamed): the step without the weight stream
            tr.zero_()
            s.engine.probe_consumers(st)
            torch.cuda.synchronize()
            tc = tr.view(-1, 128).cpu().numpy().astype(np.float64)
            Gc = int((tc[:, 0] > 0).sum())
            tc = tc[:Gc]
            rc = (tc - tc[:, 0:1]) / 100.0
            res["consumers_only_phases"] = [
                {"layer": l, "phase": nm, "median_us": float(np.median(rc[:, 2 + 12 * l + k]))}
                for l in range(min(2, args.layers)) for k, nm in enumerate(NAMES)]
            res["consumers_only_head_done_us"] = float(np.median(rc[:, 127]))
            res["consumers_only_inside"] = {
                f"L{l} {op}": {"A_in_regs": float(np.median(rc[:, 108 + 3 * (2 * l + i)])),
                               "blocks_done": float(np.median(rc[:, 109 + 3 * (2 * l + i)])),
                               "barrier_passed": float(np.median(rc[:, 110 + 3 * (2 * l + i)]))}
                for l in range(2) for i, op in enumerate(("QKV", "SwiGLU"))}
            tr.copy_(traced)
            t = tr.view(-1, 128).cpu().numpy()
            G = int((t[:, 0] > 0).sum())
            t = t[:G].astype(np.float64)
            t0 = t[:, 0:1]
            rel = (t - t0) / 100.0  # us (100 MHz)
            rows = []
            for l in range(min(8, args.layers)):
                for k, nm in enumerate(NAMES):
                    col = rel[:, 2 + 12 * l + k]
                    rows.append({"layer": l, "phase": nm, "median_us": float(np.median(col)),
                                 "max_us": float(col.max()), "min_us": float(col.min())})
            loader = [{"op": i, "median_us": float(np.median(rel[:, 100 + i])), "max_us": float(rel[:, 100 + i].max())}
                      for i in range(8)]
            res["phases"] = rows
            res["loader_op_issued"] = loader
            res["loader_end_median_us"] = float(np.median(rel[:, 120]))
            res["head_staged_median_us"] = float(np.median(rel[:, 126]))
            res["head_done_median_us"] = float(np.median(rel[:, 127]))
            res["head_done_max_us"] = float(rel[:, 127].max())
        del s
    os.environ.pop("LLJ_ENGINE", None)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1))
    print(f"engine {res['engine_us']:.1f} us/step, chain {res['chain_us']:.1f} us/step")
    prev = 0.0
    for r in res["phases"][:18]:
        print(f"L{r['layer']} {r['phase']:>13}: median {r['median_us']:8.2f} (+{r['median_us'] - prev:6.2f})  "
              f"max {r['max_us']:8.2f}")
        prev = r["median_us"]
    for r in res["loader_op_issued"]:
        print(f"loader op {r['op']} last DMA issued: median {r['median_us']:.2f} max {r['max_us']:.2f}")
    print("loader-only probe, last DMA of each op (us after the loader's start): " +
          " ".join(f"{v:.2f}" for v in res["probe_loader_op_issued"]) + f"; stream end {res['probe_stream_end_us']:.1f}; "
          f"weights in one allocation: stream end {res['probe_one_alloc_stream_end_us']:.1f}")
    prev = 0.0
    for r in res["consumers_only_phases"]:
        print(f"consumers only L{r['layer']} {r['phase']:>13}: median {r['median_us']:8.2f} (+{r['median_us'] - prev:6.2f})")
        prev = r["median_us"]
    print(f"consumers only: head done {res['consumers_only_head_done_us']:.1f} us")
    for k, v in res["consumers_only_inside"].items():
        print(f"consumers only inside {k}: " + ", ".join(f"{a} {b:.2f}" for a, b in v.items()))
    print(f"loader end {res['loader_end_median_us']:.1f}; head staged {res['head_staged_median_us']:.1f}, "
          f"head done {res['head_done_median_us']:.1f} (max {res['head_done_max_us']:.1f})")


if __name__ == "__main__":
    main()
