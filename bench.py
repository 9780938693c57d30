"""Decode throughput of the MI355X quantized LLaMA path (BASELINE.json metric).

Workload: LLaMA-7B with --quantize gptq.int4, synthetic weights of the
exact shapes (random packed int4 codes, zeros = 8, scales ~ U(0.5, 1.5) * 0.02 / 7, bf16
embeddings ~ N(0, 0.02)), batch 1, a 16-token random prompt, max_seq_length 144 (prompt +
128 new tokens), greedy decoding. One "step" = one decode token for every sequence of the
batch = one replay of the captured decode graph (embedding -> 32 fused blocks -> ln_f +
lm_head -> argmax -> next-token/position update). `value` = decode tokens/s summed over
ranks (B * K * world / max-over-ranks time of the K timed steps).

Multi-GPU: replicas only (the path is not sharded; no collective on the data
path). Every rank runs its own replica; the barrier and the max-over-ranks timing use
torch.distributed over gloo (host tensors; no RCCL communicator is created). Launch either
with python -m torch.distributed.run --nproc-per-node N bench.py --gpus N, or plainly as
bench.py --gpus N, which spawns the N replica processes itself (spawn_replicas).
The C4 leg (`c4_13b`) runs LLaMA-13B gptq.int4 batch 1 on every replica (BASELINE configs[4]).
The timed K steps are centred on position 80 where the cache allows (SURVEY §8d workload).

Also reported, on the same JSON line:
  roofline      dominant kernel (rms_2 + c_fc1/c_fc2 int4 GEMV + silu*mul, 1 launch per
                layer, 45.2 MB of algorithmic bytes at 7B) timed with HIP events on the
                stream it runs on, vs the 8 TB/s HBM peak;
  step_roofline algorithmic bytes of a whole decode step / step time;
  cpu_baseline  the numpy port of the reference's CPU path (oracle/, dequantize-every-call
                like ColBlockQuantizedLinear's fallback, quantization.py:420-421) timed on a
                bounded sample (one decode token through a few layers, scaled to 32);
  bs8           the same workload at batch 8 (aggregate tokens/s and its step roofline);
  c4_13b        BASELINE configs[4]: LLaMA-13B gptq.int4 bs=1 on every replica;
  c1_bf16       BASELINE configs[1]: LLaMA-7B bf16 (unquantized) bs=1;
  c3_int8       BASELINE configs[3]: LLaMA-7B llm.int8 bs=8 (random weights' outlier columns; `regimes`
                adds SURVEY §8d's 6 columns x20).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


# ----------------------------------------------------------------------------- distributed
def dist_init():
    """Process group from the torchrun-style environment. The replicas exchange nothing on the
    data path, so the only collectives (the barrier around the timed region and the
    max-over-ranks / sum-over-ranks of the result) run over gloo on host tensors: no RCCL
    communicator is ever created (replicas only)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        import torch.distributed as dist

        dist.init_process_group(backend="gloo")
        return dist.get_rank(), ws, int(os.environ.get("LOCAL_RANK", "0"))
    return 0, 1, 0


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_replicas(n: int, argv, timeout_s: float = 3000.0, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` started without a launcher: start N child processes of this script
    with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), one per GPU
    (LOCAL_RANK i -> cuda:i), BEFORE this process touches the GPU (it never does: only the
    children initialise HIP). All children are polled together: the first non-zero exit
    terminates the others (a replica that died would otherwise leave its siblings blocked in the
    gloo barrier) and is returned; past `timeout_s` every child is terminated and 124 returned.
    Rank 0's stdout carries the JSON line."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    t_end = time.monotonic() + timeout_s
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            print(f"[bench] a replica exited with {bad[0]}: stopping the others", file=sys.stderr)
            stop_all()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        if time.monotonic() > t_end:
            print(f"[bench] replicas still running after {timeout_s:.0f} s: stopping them", file=sys.stderr)
            stop_all()
            return 124
        time.sleep(poll_s)


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()


def aggregate(local_seconds: float, local_tokens: int, ws: int):
    """(max seconds over ranks, total tokens over ranks), over gloo on host tensors."""
    if ws == 1:
        return local_seconds, local_tokens
    import torch.distributed as dist

    t = torch.tensor([local_seconds], dtype=torch.float64)
    n = torch.tensor([float(local_tokens)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), int(n.item())


# ----------------------------------------------------------------------------- model
def build_model(name: str, mode: str, seed: int = 1234, outliers: str | None = None):
    """LLaMA `name` under quantization `mode` with synthetic weights.

    llm.int8 only, `outliers` sets the LLM.int8() outlier regime of every Linear input (the
    activation columns with some |A16| >= 6.0 that take the fp16 side product): None = the random
    weights' own (~0 in the norm outputs, a few in y, ~300 in the down-projection input h);
    "none" = no outlier column anywhere (c_attn's v rows and c_fc1 / c_fc2 scaled by 0.5 / 0.4);
    "6x20" = SURVEY §8d's regime: those scalings plus 6 columns of every Linear input made 20x larger
    (RMSNorm gains of rms_1 / rms_2 / ln_f, c_attn's v rows, c_fc1 / c_fc2 rows by sqrt(20) each)."""
    from lit_llama import LLaMA
    from lit_llama.utils import EmptyInitOnDevice

    dev = torch.device("cuda")
    with EmptyInitOnDevice(device=dev, dtype=torch.bfloat16, quantization_mode=mode):
        model = LLaMA.from_name(name)
    g = torch.Generator(device=dev).manual_seed(seed)
    with torch.no_grad():
        for mod in model.modules():
            if hasattr(mod, "quant_weight"):
                mod.quant_weight.copy_(torch.randint(0, 256, mod.quant_weight.shape, device=dev, dtype=torch.uint8,
                                                     generator=g))
                # scales U(0.5, 1.5) * 0.02 / 7, zeros 8; gptq.int8 the same at 8 bits
                half = 2 ** (mod.bits - 1)  # 8 / 128
                mod.scales.copy_((torch.rand(mod.scales.shape, device=dev, generator=g) + 0.5) * (0.02 / (half - 1)))
                mod.zeros.fill_(float(half))
            elif isinstance(mod, torch.nn.Linear):
                mod.weight.normal_(0.0, 0.02, generator=g)
            elif isinstance(mod, torch.nn.Embedding):
                mod.weight.normal_(0.0, 0.02, generator=g)
        for blk in model.transformer.h:
            blk.rms_1.scale.fill_(1.0)
            blk.rms_2.scale.fill_(1.0)
        model.transformer.ln_f.scale.fill_(1.0)
    if mode == "llm.int8":  # quantize the random bf16 weights (Linear8bitLt._quantize_weight)
        cfg = model.config
        C = cfg.n_embd
        cols = torch.arange(6, device=dev) * (C // 6) + 7  # the 6 outlier columns of every input (< C)
        for blk in model.transformer.h:
            for name_, mod in (("qkv", blk.attn.c_attn), ("o", blk.attn.c_proj), ("fc1", blk.mlp.c_fc1),
                               ("fc2", blk.mlp.c_fc2), ("down", blk.mlp.c_proj)):
                w = torch.empty((mod.out_features, mod.in_features), dtype=torch.float32, device=dev)
                w.normal_(0.0, 0.02, generator=g)
                if outliers in ("none", "6x20"):
                    if name_ == "qkv":
                        w[2 * C:] *= 0.5  # v: attention outputs y below 6
                    elif name_ in ("fc1", "fc2"):
                        w *= 0.4  # h = silu(a1) a2 below 6
                    if outliers == "6x20":
                        if name_ == "qkv":
                            w[2 * C + cols] *= 20.0  # y columns 20x
                        elif name_ in ("fc1", "fc2"):
                            w[cols] *= 20.0 ** 0.5  # h columns 20x
                mod._quantize_weight(w.to(torch.bfloat16))
        w = torch.empty((model.lm_head.out_features, C), dtype=torch.bfloat16, device=dev)
        w.normal_(0.0, 0.02, generator=g)
        model.lm_head._quantize_weight(w)
        if outliers == "6x20":
            with torch.no_grad():
                for norm in [b.rms_1 for b in model.transformer.h] + [b.rms_2 for b in model.transformer.h] + \
                        [model.transformer.ln_f]:
                    norm.scale[cols] = 20.0
    elif outliers is not None:
        raise ValueError("outlier regimes are an llm.int8 setting")
    return model.eval()


def weight_bytes(model) -> int:
    """Algorithmic weight bytes streamed per decode step (every Linear once; wte excluded:
    only gathered rows count). int4: packed codes + (scale, zero) per row as stored on the
    reference side (bf16 each)."""
    total = 0
    for mod in model.modules():
        if hasattr(mod, "quant_weight"):
            total += mod.quant_weight.numel() + 2 * mod.out_features * 2
        elif hasattr(mod, "SCB"):
            total += mod.weight.numel() + 4 * mod.out_features
        elif isinstance(mod, torch.nn.Linear):
            total += mod.weight.numel() * 2
    return total


def step_bytes(model, B: int, pos_mean: float) -> float:
    """W + sum_b KV_read(p_b) + B*KV_write + B*C*2 (embedding row)."""
    cfg = model.config
    kv_per_tok = 2 * cfg.n_layer * cfg.n_embd * 2  # k and v, bf16, all layers
    return weight_bytes(model) + B * kv_per_tok * (pos_mean + 1) + B * kv_per_tok + B * cfg.n_embd * 2


# ----------------------------------------------------------------------------- timing
POS_CENTER = 80  # a 128-token generation after a 16-token prompt has mean position 80


def untimed_steps(prompt_len: int, S: int, warmup: int, steps: int) -> int:
    """Decode steps before the timed region: at least `warmup`, and enough that the K timed
    steps are centred on position POS_CENTER (the §8d workload) when the cache allows it."""
    centred = POS_CENTER - prompt_len - steps // 2
    room = S - prompt_len - 1 - steps  # the timed steps must stay inside the S-slot cache
    return max(warmup, min(centred, room))


def time_decode(model, B, prompt_len, S, warmup, steps, ws, seed=1234, use_graph=True):
    from lit_llama.engine import DecodeSession

    cfg = model.config
    skip = untimed_steps(prompt_len, S, warmup, steps)
    total = prompt_len + 1 + skip + steps
    assert total <= cfg.block_size, "positions beyond block_size"
    g = torch.Generator().manual_seed(seed)
    prompts = torch.randint(3, cfg.vocab_size, (B, prompt_len), generator=g).cuda()
    sess = DecodeSession(model, B, S, total, use_graph=use_graph)
    sess.prefill(prompts)  # one-time work (int4 repack, kernel attributes) stays out of the timings
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sess.prefill(prompts)
    torch.cuda.synchronize()
    t_prefill = time.perf_counter() - t0
    sess.capture()
    if skip:
        sess.decode(skip)
    barrier(ws)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    sess.decode(steps)
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier(ws)
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    # the step that reads position p writes slot p and attends p + 1 keys; the first timed
    # step runs at position prompt_len + skip
    pos_mean = prompt_len + skip + (steps - 1) / 2.0
    return dict(seconds=max(wall, gpu_s), gpu_seconds=gpu_s, wall_seconds=wall, t_prefill=t_prefill,
                pos_mean=pos_mean, tokens=B * steps, session=sess)


def time_stub(steps, warmup, ws, step_s=1e-3):
    """--stub: the replica / timing / aggregation plumbing without a GPU (CPU rehearsal of
    `bench.py --gpus N`); one 'step' is a sleep. Never a measurement."""
    for _ in range(warmup):
        time.sleep(step_s)
    barrier(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        time.sleep(step_s)
    wall = time.perf_counter() - t0
    barrier(ws)
    return dict(seconds=wall, tokens=steps)


def time_dominant_kernel(model, B, iters=10):
    """Average duration of the fused rms_2 + c_fc1/c_fc2 (+silu*mul) launch, one launch per
    layer on that layer's weights (no cache reuse between consecutive launches: 32 x 45 MB),
    measured with HIP events on the launch stream."""
    from lit_llama import _hip
    from lit_llama.model import MLP, _wspec

    cfg = model.config
    C, H = cfg.n_embd, MLP.hidden(cfg)
    x = torch.randn(B, C, device="cuda").to(torch.bfloat16)
    h = torch.empty(B, H, device="cuda", dtype=torch.bfloat16)
    specs = []
    for blk in model.transformer.h:
        (f1, w1, s1), (f2, w2, s2) = _wspec(blk.mlp.c_fc1), _wspec(blk.mlp.c_fc2)
        specs.append((f1, blk.rms_2, w1, s1, w2, s2))
    st = _hip.stream()

    def run_all():
        for f1, rms, w1, s1, w2, s2 in specs:
            _hip.call("llj_norm_swiglu", f1, x.data_ptr(), rms.scale.data_ptr(), rms.eps, w1.data_ptr(), _hip.ptr(s1),
                      w2.data_ptr(), _hip.ptr(s2), h.data_ptr(), B, H, C, None, 0, None, None, 0, st)

    run_all()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        run_all()
    ev1.record()
    torch.cuda.synchronize()
    avg_s = ev0.elapsed_time(ev1) / 1e3 / (iters * len(specs))
    f1, _, w1, s1, w2, s2 = specs[0]
    wbytes = 2 * (w1.numel() * w1.element_size()) + 2 * 2 * (H * 2)  # two matrices + (scale, zero) bf16
    abytes = wbytes + B * C * 2 + B * H * 2 + C * 2  # + x row(s), h row(s), norm weight
    return avg_s, abytes


# the dominant decode launch (W4, fused RMSNorm, SwiGLU; 4 waves, 2 chunks in flight, one row)
DOMINANT = "llj::gemv_kernel<0, 2, 3, 4, 2, 1, 1>"


def graph_kernel_us(kernel_prefix: str = "void " + DOMINANT):
    """In-graph average duration of the dominant launch from the newest committed kernel trace of
    the decode graph alone: profiles/<round>_graph_kernel_stats.csv, the rocprofv3 --kernel-trace
    --stats summary of `bench.py --decode-only` (graph replays only: no isolated loop in the
    process, so the average is over launches inside the captured chain). None when absent."""
    import csv

    best = None
    for p in sorted((REPO / "profiles").glob("r*_graph_kernel_stats.csv")):
        try:
            with open(p) as f:
                for r in csv.DictReader(f):
                    if r["Name"].startswith(kernel_prefix):
                        best = (float(r["AverageNs"]) / 1e3, p.name)
        except (OSError, KeyError, ValueError):
            continue
    return best


def achievable_read_gbs(gb: float = 4.0, iters: int = 5):
    """The achievable HBM read rate: llj_stream_read (non-temporal 16 B loads, grid-stride) over a
    `gb` GB buffer (16x the 256 MB MALL, so the reads come from HBM), best over a few grid sizes,
    HIP events on the launch stream. The denominator beside the 8 TB/s spec."""
    from lit_llama import _hip

    n = int(gb * 1e9) // 16 * 16
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    buf.fill_(1)
    out = torch.empty(65536, dtype=torch.float32, device="cuda")
    st = _hip.stream()
    best = 0.0
    for grid in (2048, 4096, 8192):
        _hip.call("llj_stream_read", buf.data_ptr(), n, out.data_ptr(), grid, st)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(iters):
            _hip.call("llj_stream_read", buf.data_ptr(), n, out.data_ptr(), grid, st)
        ev1.record()
        torch.cuda.synchronize()
        best = max(best, n * iters / (ev0.elapsed_time(ev1) / 1e3) / 1e9)
    del buf
    torch.cuda.empty_cache()
    return best


def pmc_traffic(kernel_prefix: str = DOMINANT):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary:
    profiles/<round>_pmc_summary.json (tools/profile_summary.py over separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of the 7B gptq.int4 bs=1 decode, gfx950 correction
    2*FETCH+WRITE KiB), else the round-1 profiles/<round>_summary.json. None when absent."""
    best = None
    for p in sorted((REPO / "profiles").glob("r*_pmc_summary.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        for name, k in d.get("kernels", {}).items():
            e = k.get("bs1", {})
            if name.startswith(kernel_prefix) and "hbm_bytes" in e:
                best = (e["hbm_bytes"], p.name, e.get("profiled_us"))
    if best:
        return best
    for p in sorted((REPO / "profiles").glob("r*_summary.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        for name, lp in d.get("dominant_loop", {}).items():
            if name.startswith(kernel_prefix[:-8]) and "hbm_bytes_per_dispatch" in lp:
                best = (lp["hbm_bytes_per_dispatch"], p.name, lp.get("avg_us"))
    return best


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(model, budget_s: float = 20.0):
    """The oracle's numpy port of the reference CPU decode path (dequantize every call),
    one decode token at position 80 through n sampled layers + lm_head, scaled to the full
    depth. Threads: numpy/BLAS limited to 16 (the box's CPU share)."""
    from threadpoolctl import threadpool_limits

    from oracle import llama_np as O

    cfg = model.config
    C, nh = cfg.n_embd, cfg.n_head
    hs = C // nh
    p = 80
    rng = np.random.default_rng(0)

    def lin_np(mod):
        return (mod.quant_weight.cpu().numpy(), mod.scales.float().cpu().numpy(), mod.zeros.float().cpu().numpy())

    def qlin(x, spec):  # ColBlockQuantizedLinear CPU fallback: get_weight + F.linear per call
        W = O.colblock_get_weight(*spec, 4)
        return x @ W.T

    rope = O.build_rope_cache(cfg.block_size, hs)
    threads = 16
    with threadpool_limits(limits=threads):
        layer_times = []
        t_start = time.perf_counter()
        x = rng.standard_normal((1, 1, C)).astype(np.float32) * 0.02
        for li, blk in enumerate(model.transformer.h):
            specs = [lin_np(m) for m in (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc1, blk.mlp.c_fc2, blk.mlp.c_proj)]
            kc = rng.standard_normal((1, nh, p + 1, hs)).astype(np.float32)
            vc = rng.standard_normal((1, nh, p + 1, hs)).astype(np.float32)
            t0 = time.perf_counter()
            h = O.rmsnorm(x, np.ones(C, np.float32))
            qkv = qlin(h, specs[0])
            q = O.apply_rope(qkv[..., :C].reshape(1, 1, nh, hs), rope[p:p + 1]).transpose(0, 2, 1, 3)
            k = O.apply_rope(qkv[..., C:2 * C].reshape(1, 1, nh, hs), rope[p:p + 1]).transpose(0, 2, 1, 3)
            kc[:, :, p] = k[:, :, 0]
            vc[:, :, p] = qkv[..., 2 * C:].reshape(1, nh, hs)
            att = (q @ kc.transpose(0, 1, 3, 2)) / math.sqrt(hs)
            att = np.exp(att - att.max(-1, keepdims=True))
            att /= att.sum(-1, keepdims=True)
            y = (att @ vc).transpose(0, 2, 1, 3).reshape(1, 1, C)
            x = x + qlin(y, specs[1])
            h = O.rmsnorm(x, np.ones(C, np.float32))
            m = O.silu(qlin(h, specs[2])) * qlin(h, specs[3])
            x = x + qlin(m, specs[4])
            layer_times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > budget_s * 0.6 and len(layer_times) >= 1:
                break
        t0 = time.perf_counter()
        qlin(O.rmsnorm(x, np.ones(C, np.float32)), lin_np(model.lm_head))
        t_head = time.perf_counter() - t0
    per_layer = float(np.mean(layer_times))
    t_tok = per_layer * cfg.n_layer + t_head
    return {"value": 1.0 / t_tok, "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"1 decode token (bs=1, position {p}) through {len(layer_times)} of {cfg.n_layer} layers "
                      f"({per_layer:.2f} s/layer) + lm_head ({t_head:.2f} s), scaled to {cfg.n_layer} layers; "
                      "numpy port of the reference CPU path with per-call int4 dequantization"}


# ----------------------------------------------------------------------------- main
def c4_leg(args, ws):
    """C4 (BASELINE.json configs[4]): LLaMA-13B gptq.int4, batch 1, one replica per GPU; every
    rank decodes its own sequence and `value` sums over the ranks."""
    m13 = build_model("13B", "gptq.int4")
    r = time_decode(m13, 1, args.prompt_len, args.max_seq_length, args.warmup, args.steps, ws)
    t, tok = aggregate(r["seconds"], r["tokens"], ws)
    sb = step_bytes(m13, 1, r["pos_mean"])
    out = {"workload": "LLaMA-13B --quantize gptq.int4 greedy decode, batch 1 per replica",
           "value": round(tok / t, 2), "unit": "tokens/s", "n_replicas": ws,
           "ms_per_step": round(t / args.steps * 1e3, 4),
           "step_roofline_frac": round(sb / (r["seconds"] / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}
    del r["session"], m13
    torch.cuda.empty_cache()
    return out


def config_leg(args, ws, name: str, mode, B: int, outliers=None, workload: str = ""):
    """One more BASELINE.json config on the same replicas and timing as the headline: C1 (LLaMA-7B
    bf16, bs=1; reference generate.py:121 bf16-true) and C3 (LLaMA-7B llm.int8, bs=8, reference
    quantization.py:36-75) in the outlier regimes of build_model. The model is built, timed and freed
    here, so the legs never hold two 7B models at once."""
    import gc

    m = build_model(name, mode, outliers=outliers)
    r = time_decode(m, B, args.prompt_len, args.max_seq_length, args.warmup, args.steps, ws)
    t, tok = aggregate(r["seconds"], r["tokens"], ws)
    sb = step_bytes(m, B, r["pos_mean"])
    out = {"workload": workload, "value": round(tok / t, 2), "unit": "tokens/s", "n_replicas": ws, "batch": B,
           "ms_per_step": round(t / args.steps * 1e3, 4),
           "step_roofline_frac": round(sb / (r["seconds"] / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}
    del r["session"], m
    gc.collect()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="7B")
    ap.add_argument("--quantize", default="gptq.int4", choices=["gptq.int4", "llm.int8", "none"])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt-len", type=int, default=16)
    ap.add_argument("--max-seq-length", type=int, default=144)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-bs8", action="store_true")
    ap.add_argument("--no-c4", action="store_true", help="skip the LLaMA-13B replica leg (C4)")
    ap.add_argument("--no-configs", action="store_true", help="skip the C1 (7B bf16 bs=1) and C3 (7B llm.int8 bs=8) legs")
    ap.add_argument("--only-dominant", action="store_true",
                    help="profiling aid: only the dominant-kernel loop (for the PMC traffic passes)")
    ap.add_argument("--decode-only", action="store_true",
                    help="profiling aid: only the timed decode (graph replays), printed as a short line")
    ap.add_argument("--eager", action="store_true",
                    help="profiling aid: decode steps launched one by one instead of graph replays (PMC passes)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU rehearsal of the replica launch / timing / aggregation (no GPU, no measurement)")
    ap.add_argument("--stub-fail-rank", type=int, default=-1,
                    help="with --stub: this rank exits 3 before the barrier (launcher failure test)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start one replica process per GPU before anything touches the GPU
        sys.exit(spawn_replicas(args.gpus, sys.argv[1:]))
    rank, ws, local_rank = dist_init()
    if ws != args.gpus:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE {ws}", file=sys.stderr)

    if args.stub:
        if args.stub_fail_rank == rank:  # launcher test: this replica dies before the barrier
            sys.exit(3)
        r = time_stub(args.steps, args.warmup, ws)
        t_max, tokens = aggregate(r["seconds"], r["tokens"], ws)
        if rank == 0:
            print(json.dumps({"metric": "stub (plumbing rehearsal, not a measurement)", "value": tokens / t_max,
                              "unit": "steps/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                              "ms_per_step": t_max / args.steps * 1e3, "stub": True,
                              "config": {"parallelism": f"replicas x{ws}"}}), flush=True)
        if ws > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
        return

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    mode = None if args.quantize == "none" else args.quantize
    model = build_model(args.model, mode)
    S = args.max_seq_length

    if args.only_dominant:
        k_s, k_bytes = time_dominant_kernel(model, args.batch)
        print(json.dumps({"dominant_avg_us": round(k_s * 1e6, 2), "bytes_per_launch": k_bytes}), flush=True)
        return
    r = time_decode(model, args.batch, args.prompt_len, S, args.warmup, args.steps, ws, use_graph=not args.eager)
    t_max, tokens = aggregate(r["seconds"], r["tokens"], ws)
    if args.decode_only:
        if rank == 0:
            print(json.dumps({"decode_only": True, "tokens_per_s": round(tokens / t_max, 2),
                              "ms_per_step": round(t_max / args.steps * 1e3, 4)}), flush=True)
        return
    value = tokens / t_max
    ms_per_step = t_max / args.steps * 1e3
    sb = step_bytes(model, args.batch, r["pos_mean"])
    step_gbs = sb / (r["seconds"] / args.steps) / 1e9
    mem = {"max_reserved_gb": round(torch.cuda.max_memory_reserved() / 1e9, 3),
           "max_allocated_gb": round(torch.cuda.max_memory_allocated() / 1e9, 3),
           "reference_gb": "~5 (README.md:108, 7B gptq.int4)"}

    k_s, k_bytes = time_dominant_kernel(model, args.batch)
    k_gbs = k_bytes / k_s / 1e9
    in_graph = graph_kernel_us()
    ach = achievable_read_gbs()

    pmc = pmc_traffic()
    bs8 = None
    if not args.no_bs8 and args.batch != 8:
        del r["session"]
        r8 = time_decode(model, 8, args.prompt_len, S, args.warmup, args.steps, ws)
        t8, tok8 = aggregate(r8["seconds"], r8["tokens"], ws)
        sb8 = step_bytes(model, 8, r8["pos_mean"])
        bs8 = {"value": tok8 / t8, "unit": "tokens/s", "ms_per_step": t8 / args.steps * 1e3,
               "step_roofline_frac": sb8 / (r8["seconds"] / args.steps) / 1e9 / HBM_PEAK_GBS}
        del r8["session"]

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and mode == "gptq.int4":
        cpu = cpu_baseline(model)

    c4 = c1 = c3 = None
    legs = args.model == "7B" and mode == "gptq.int4"
    r.pop("session", None)  # the headline's numbers stay in r; its graph and cache are freed
    if legs:
        del model
        import gc

        gc.collect()
        torch.cuda.empty_cache()
    if not args.no_c4 and legs:
        c4 = c4_leg(args, ws)
    if not args.no_configs and legs:
        c1 = config_leg(args, ws, "7B", None, 1,
                        workload="LLaMA-7B bf16 (unquantized) greedy decode, batch 1 per replica (BASELINE configs[1])")
        c3 = config_leg(args, ws, "7B", "llm.int8", 8,
                        workload="LLaMA-7B --quantize llm.int8 greedy decode, batch 8 per replica (BASELINE configs[3]); "
                                 "outlier columns: the random weights' own")
        c3["regimes"] = {"6x20": config_leg(args, ws, "7B", "llm.int8", 8, outliers="6x20",
                                            workload="C3 with SURVEY 8d's regime: 6 columns of every Linear input x20")}

    if rank == 0:
        name = {"gptq.int4": "gptq.int4", "llm.int8": "llm.int8", "none": "bf16"}[args.quantize]
        head7 = args.batch == 1 and mode == "gptq.int4" and args.model == "7B"
        line = {
            "metric": f"decode tokens/sec LLaMA-{args.model} {name} bs={args.batch}, 1xMI355X per replica",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "weights": {"gptq.int4": "int4 (per-row scale/zero)", "llm.int8": "int8 (LLM.int8)",
                        "none": "bf16"}[args.quantize],
            "data": "synthetic (random weights of the exact shapes, random 16-token prompts)",
            "config": {"workload": f"LLaMA-{args.model} --quantize {args.quantize} greedy decode, batch {args.batch}, "
                                   f"prompt {args.prompt_len}, max_seq_length {S}",
                       "batch_per_gpu": args.batch, "prompt_len": args.prompt_len, "max_seq_length": S,
                       "timed_positions_mean": r["pos_mean"],
                       "parallelism": f"replicas x{ws} (no collective on the data path)"},
            "roofline": {"bound": "hbm", "achieved": round(k_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(k_gbs / HBM_PEAK_GBS, 4),
                         "achievable": round(ach, 1), "frac_of_achievable": round(k_gbs / ach, 4),
                         "achievable_source": "llj_stream_read over 4 GB (measured in this run)",
                         "traffic": round(pmc[0]) if pmc and head7 else None,
                         "traffic_source": (f"profiles/{pmc[1]} (PMC FETCH_SIZE/WRITE_SIZE passes, "
                                            f"profiled {pmc[2]:.2f} us)" if pmc and head7 else None),
                         "kernel": "gemv_kernel<W4,NORM,SWIGLU> (rms_2 + c_fc1/c_fc2 + silu*mul)",
                         "bytes_per_launch": k_bytes, "avg_launch_us": round(k_s * 1e6, 2),
                         **({"in_graph_avg_launch_us": round(in_graph[0], 2),
                             "in_graph_frac": round(k_bytes / (in_graph[0] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                             "in_graph_source": f"profiles/{in_graph[1]} (rocprofv3 kernel trace of bench.py --decode-only)"}
                            if in_graph and head7 else {})},
            "decode_path": "launch chain (5 fused launches per layer)",
            "step_roofline": {"bytes_per_step": sb, "achieved": round(step_gbs, 1), "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                              "frac_of_achievable": round(step_gbs / ach, 4)},
            "reference_formula_tokens_per_s": round(r["tokens"] / (r["seconds"] + r["t_prefill"]), 2),
            "memory": mem,
            "cpu_baseline": cpu,
            "bs8": bs8,
            "c4_13b": c4,
            "c1_bf16": c1,
            "c3_int8": c3,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
