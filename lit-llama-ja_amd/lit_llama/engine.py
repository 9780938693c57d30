"""Decode session: the reference's token loop (generate.py:61-87) with the per-token work
captured once into a HIP graph.

One decode step = embedding of the current token (which also advances the device-side
position), the n_layer fused blocks, ln_f + lm_head and the next-token choice -- the greedy
argmax (top_k = 1) or the temperature / top-k sampler (llj_sample, generate.py:66-74; its
uniform comes from a counter hash of (seed, position, row), or from a caller's table of
uniforms per position) -- which writes the next token both into `cur` and into the output id
buffer. Nothing in the step reads the host, so replaying the graph K times generates K tokens
with no host round trip (the reference syncs per layer at model.py:221 and per token at
generate.py:86).

Batch B > 1 decodes B equal-length prompts together (each row equals an independent B=1
run: tests/test_model_gpu.py); the reference's generate() is batch 1 only (generate.py:62).

Batch 1 with int4 (gptq.int4) weights and a cache of at most ENGINE_MAX_S slots runs each step as
ONE launch of the persistent decode engine (csrc/engine.hip, llj_engine_step): the same step with
the weight stream carried across every op edge and the op outputs handed between CUs in-launch.
Other configurations (and LLJ_ENGINE=0) keep the fused launch chain.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _hip
from .model import LLaMA, MLP, QKV_ROWS, _Work

# caches up to this many slots take the persistent engine (its attention runs one head per CU; past
# this length the launch chain's split-K attention spreads a head over more CUs)
ENGINE_MAX_S = 512
# on by default only once it beats the launch chain on the bench workload (LLJ_ENGINE=1 / 0 override)
ENGINE_DEFAULT = "0"


class _EngLayer(ctypes.Structure):  # include/lit_llama_amd.h llj_engine_layer
    _fields_ = [(n, ctypes.c_void_p) for n in ("w_qkv", "sz_qkv", "w_o", "sz_o", "w_fc1", "sz_fc1", "w_fc2", "sz_fc2",
                                               "w_down", "sz_down", "rms1", "rms2", "kcache", "vcache")] + \
               [("eps1", ctypes.c_float), ("eps2", ctypes.c_float)]


class _EngPlan(ctypes.Structure):  # include/lit_llama_amd.h llj_engine_plan
    _fields_ = [("layers", ctypes.c_void_p)] + [(n, ctypes.c_int) for n in ("n_layer", "C", "H", "V", "n_head", "S")] + \
               [("wte", ctypes.c_void_p), ("ln_f", ctypes.c_void_p), ("eps_f", ctypes.c_float),
                ("w_head", ctypes.c_void_p), ("sz_head", ctypes.c_void_p), ("rope", ctypes.c_void_p),
                ("pos", ctypes.c_void_p), ("cur", ctypes.c_void_p), ("tokens", ctypes.c_void_p),
                ("logits", ctypes.c_void_p), ("arena", ctypes.c_void_p), ("flags", ctypes.c_int),
                ("grid", ctypes.c_int), ("ring_blocks", ctypes.c_int), ("trace", ctypes.c_void_p)]


def engine_supported(model: LLaMA, specs, batch: int, S: int) -> str | None:
    """None if the persistent engine takes this decode session, else why not."""
    if os.environ.get("LLJ_ENGINE", ENGINE_DEFAULT) == "0":
        return "disabled (LLJ_ENGINE=0)"
    cfg = model.config
    hs = cfg.n_embd // cfg.n_head
    if model._generic():
        return "any-shape / fp32 path"
    if batch != 1:
        return "batch > 1"
    if S > ENGINE_MAX_S:
        return f"cache of {S} slots > {ENGINE_MAX_S}"
    if hs not in (64, 128) or cfg.n_embd % 128 or MLP.hidden(cfg) % 128 or cfg.padded_vocab_size % 16:
        return "shape"
    if cfg.padded_vocab_size > 65536:
        return "vocabulary > 65536"
    cus = torch.cuda.get_device_properties(model.transformer.wte.weight.device).multi_processor_count
    if cfg.n_embd // 16 > cus:  # one QKV unit (head, 16-dim slice) per CU (13B: 320 units > 256 CUs)
        return f"{cfg.n_embd // 16} QKV units > {cus} CUs"
    if cfg.n_embd > 4480:  # the K = C ops keep their A fragments in registers (csrc/engine.hip AREG_C)
        return "n_embd > 4480"
    fmts = {sp[0] for layer in specs["layers"] for sp in layer} | {specs["head"][0]}
    if fmts != {0}:
        return "not every Linear is per-row int4 (W4P)"
    mods = [m for blk in model.transformer.h for m in (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc1, blk.mlp.c_fc2,
                                                       blk.mlp.c_proj)] + [model.lm_head]
    if any(getattr(m, "bias", None) is not None for m in mods):
        return "biased Linear"
    L = _hip.lib()
    if L.llj_engine_ring_blocks(cfg.n_embd, MLP.hidden(cfg), cfg.n_head) < 80:
        return "LDS"
    return None


class _Engine:
    """Device plan of the persistent decode engine for one session (batch 1)."""

    def __init__(self, model: LLaMA, specs, sess: "DecodeSession", greedy: bool):
        cfg = model.config
        C, H, V = cfg.n_embd, MLP.hidden(cfg), cfg.padded_vocab_size
        dev = sess.dev
        L = _hip.lib()
        lay = (_EngLayer * cfg.n_layer)()
        self.keep = []  # tensors whose pointers the plan holds
        for i, blk in enumerate(model.transformer.h):
            (_, wa, sa), (_, wp, sp), (_, w1, s1), (_, w2, s2), (_, wd, sd) = specs["layers"][i]
            kc, vc = model.kv_caches[i]
            e = lay[i]
            e.w_qkv, e.sz_qkv, e.w_o, e.sz_o = wa.data_ptr(), sa.data_ptr(), wp.data_ptr(), sp.data_ptr()
            e.w_fc1, e.sz_fc1, e.w_fc2, e.sz_fc2 = w1.data_ptr(), s1.data_ptr(), w2.data_ptr(), s2.data_ptr()
            e.w_down, e.sz_down = wd.data_ptr(), sd.data_ptr()
            e.rms1, e.rms2 = blk.rms_1.scale.data_ptr(), blk.rms_2.scale.data_ptr()
            e.kcache, e.vcache = kc.data_ptr(), vc.data_ptr()
            e.eps1, e.eps2 = float(blk.rms_1.eps), float(blk.rms_2.eps)
            self.keep += [wa, sa, wp, sp, w1, s1, w2, s2, wd, sd, kc, vc]
        raw = torch.frombuffer(bytearray(bytes(lay)), dtype=torch.uint8)
        self.layers = raw.to(dev)
        self.arena = torch.zeros(L.llj_engine_arena_bytes(C, H), dtype=torch.uint8, device=dev)
        fh, wh, sh = specs["head"]
        self.keep += [wh, sh]
        rope = model.rope_cache
        assert rope.dtype == torch.float32 and rope.is_contiguous()
        P = _EngPlan()
        P.layers = self.layers.data_ptr()
        P.n_layer, P.C, P.H, P.V, P.n_head, P.S = cfg.n_layer, C, H, V, cfg.n_head, sess.S
        P.wte = model.transformer.wte.weight.data_ptr()
        P.ln_f, P.eps_f = model.transformer.ln_f.scale.data_ptr(), float(model.transformer.ln_f.eps)
        P.w_head, P.sz_head = wh.data_ptr(), sh.data_ptr()
        P.rope = rope.data_ptr()
        P.pos, P.cur, P.tokens = sess.pos.data_ptr(), sess.cur.data_ptr(), sess.tokens.data_ptr()
        P.logits, P.arena = sess.logits.data_ptr(), self.arena.data_ptr()
        P.flags = 1 if greedy else 0
        P.grid = 0
        P.ring_blocks = L.llj_engine_ring_blocks(C, H, cfg.n_head)
        P.trace = None
        self.plan = P
        self.trace = None

    def enable_trace(self, grid: int = 1024) -> torch.Tensor:
        """Profiling only: per-CU phase stamps (s_memrealtime, 100 MHz) of the following steps,
        csrc/engine.hip STAMP_* indices; capture the graph after enabling."""
        self.trace = torch.zeros(grid * 128, dtype=torch.int64, device=self.arena.device)
        self.plan.trace = self.trace.data_ptr()
        return self.trace

    def probe_stream(self, st) -> None:
        """Profiling only: one launch in which the loader streams the whole step's weights with
        no consumers (flow control off, no step state touched): the in-engine stream rate."""
        self.plan.flags |= 2
        try:
            self.step(st)
        finally:
            self.plan.flags &= ~2

    def probe_consumers(self, st) -> None:
        """Profiling only: one step with every ring block taken as landed and nothing streamed --
        the consumers' and edges' own time. Results and the session's state are invalid after."""
        self.plan.flags |= 4
        try:
            self.step(st)
        finally:
            self.plan.flags &= ~4

    def step(self, st) -> None:
        rc = _hip.lib().llj_engine_step(ctypes.byref(self.plan), st)
        if rc != 0:
            raise _hip.HipError(f"llj_engine_step failed: {'EINVAL' if rc == 1000 else f'hipError {rc}'}")

    def error_bits(self) -> int:
        """Control word 2 behind the granules: nonzero after a step whose in-launch wait timed out."""
        cfg_words = self.arena[-64:].view(torch.int32)
        return int(cfg_words[2].item())


class DecodeSession:
    def __init__(self, model: LLaMA, batch: int, max_seq_length: int, total_len: int, use_graph: bool = True,
                 temperature: float = 1.0, top_k: int | None = 1, seed: int = 0,
                 uniforms: torch.Tensor | None = None):
        """top_k == 1: greedy; otherwise sampling at `temperature` over the top_k logits (None:
        all). uniforms: optional (total_len, batch) fp32 device table, row p = the uniforms of the
        token at position p (tests replay a reference run's draws)."""
        cfg = model.config
        assert max_seq_length <= cfg.block_size
        self.model, self.B, self.S, self.total = model, batch, max_seq_length, total_len
        dev = model.transformer.wte.weight.device
        _hip.require_device(model.transformer.wte.weight, "model")
        self.dev = dev
        if batch > QKV_ROWS:
            raise ValueError(f"decode batch {batch} > {QKV_ROWS} rows per fused launch")
        self.cur = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.pos = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tokens = torch.zeros(batch, total_len, dtype=torch.int32, device=dev)
        self.logits = torch.empty(batch, cfg.padded_vocab_size, dtype=model.act_dtype(), device=dev)
        self.use_graph = use_graph
        self.graph = None
        self.t_prompt = 0
        self.steps_done = 0
        self.specs = None
        self.work = None
        self.engine = None
        self.temperature = float(temperature)
        self.top_k = 0 if top_k is None else int(top_k)
        self.seed = int(seed) & ((1 << 64) - 1)
        if uniforms is not None:
            assert uniforms.dtype == torch.float32 and uniforms.shape == (total_len, batch) and uniforms.is_contiguous()
            _hip.require_device(uniforms, "uniforms")
        self.uniforms = uniforms

    def _choose(self, st):
        """next token of every row from self.logits -> cur and tokens[:, pos + 1]"""
        cfg = self.model.config
        if self.logits.dtype == torch.float32:  # the fp32 model (any-shape path): greedy only
            if self.top_k != 1:
                raise NotImplementedError("sampling (top_k != 1) over float32 logits: use a bfloat16 model")
            _hip.call("llj_g_argmax", self.logits.data_ptr(), self.logits.stride(0), self.B, cfg.padded_vocab_size,
                      self.cur.data_ptr(), self.tokens.data_ptr(), self.total, self.pos.data_ptr(), st)
        elif self.top_k == 1:
            _hip.call("llj_argmax", self.logits.data_ptr(), self.logits.stride(0), self.B, cfg.padded_vocab_size,
                      self.cur.data_ptr(), self.tokens.data_ptr(), self.total, self.pos.data_ptr(), st)
        else:
            _hip.call("llj_sample", self.logits.data_ptr(), self.logits.stride(0), self.B, cfg.padded_vocab_size,
                      self.temperature, self.top_k, _hip.ptr(self.uniforms), self.seed, self.cur.data_ptr(),
                      self.tokens.data_ptr(), self.total, self.pos.data_ptr(), st)

    # -- prefill: eager (rows = B*T); fills the caches, picks the first new token
    @torch.no_grad()
    def prefill(self, prompts: torch.Tensor) -> None:
        m = self.model
        B, T = prompts.shape
        assert B == self.B and T + 1 <= self.total
        m.reset_cache()
        m.kv_caches = m._alloc_kv(B, self.S, self.dev)
        if m.rope_cache is None:
            m.rope_cache = m.build_rope_cache(prompts)
        pos = torch.arange(T, device=self.dev, dtype=torch.int32)
        m._run(prompts.to(self.dev), pos, self.S, m.kv_caches, last_only_out=self.logits)
        st = _hip.stream()
        self.tokens[:, :T] = prompts.to(torch.int32)
        self.pos.fill_(T - 1)
        self._choose(st)
        self.t_prompt = T
        self.steps_done = 1
        # decode-step operands (fixed for the session)
        self.specs = m._layer_specs()
        if m._generic():  # the any-shape kernels (csrc/generic.hip)
            self.work = _Work(m.config, B, self.dev, False, self.S, generic=True, dtype=m.act_dtype())
        else:
            need_i8 = any(s[0] == 2 for layer in self.specs["layers"] for s in layer) or self.specs["head"][0] == 2
            self.work = _Work(m.config, B, self.dev, need_i8, self.S)
        self.graph = None  # the caches / operands may have changed
        why = engine_supported(m, self.specs, B, self.S)
        self.engine = _Engine(m, self.specs, self, greedy=self.top_k == 1) if why is None else None
        self.engine_off_reason = why

    def _step(self):
        m, w, B = self.model, self.work, self.B
        cfg = m.config
        st = _hip.stream()
        if self.engine is not None:  # the whole step in one launch (greedy choice included)
            self.engine.step(st)
            if self.top_k != 1:
                _hip.call("llj_sample", self.logits.data_ptr(), self.logits.stride(0), self.B, cfg.padded_vocab_size,
                          self.temperature, self.top_k, _hip.ptr(self.uniforms), self.seed, self.cur.data_ptr(),
                          self.tokens.data_ptr(), self.total, self.pos.data_ptr(), st)
            return
        if w.generic:
            _hip.call("llj_g_embedding", self.cur.data_ptr(), m.transformer.wte.weight.data_ptr(), w.x.data_ptr(), B,
                      cfg.n_embd, self.pos.data_ptr(), w.dt, st)
        else:
            _hip.call("llj_embedding", self.cur.data_ptr(), m.transformer.wte.weight.data_ptr(), w.x.data_ptr(), B,
                      cfg.n_embd, self.pos.data_ptr(), st)
        m._blocks(w, self.specs, m.kv_caches, self.pos, B, 1, self.S, st)
        m._head(w.x, B, self.specs, self.logits, st, w)
        self._choose(st)

    def capture(self):
        if self.graph is not None or not self.use_graph:
            return
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step()
        self.graph = g

    @torch.no_grad()
    def decode(self, n: int) -> None:
        """Generate n more tokens per row (positions t_prompt + steps_done ...)."""
        assert self.t_prompt + self.steps_done + n <= self.total, "beyond the output buffer"
        assert self.t_prompt + self.steps_done + n - 1 <= self.model.config.block_size, "beyond block_size"
        if self.use_graph:
            self.capture()
            for _ in range(n):
                self.graph.replay()
        else:
            for _ in range(n):
                self._step()
        self.steps_done += n

    def output(self) -> torch.Tensor:
        if self.engine is not None and self.engine.error_bits():
            raise _hip.HipError("persistent decode engine: an in-launch wait timed out (results invalid)")
        return self.tokens[:, :self.t_prompt + self.steps_done]
