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
run: tests/test_model_gpu.py); the reference's generate() is batch 1 only (generate.py:62). Up to 8
rows share every fused launch; larger batches take the ops in row slices.
"""
from __future__ import annotations

import torch

from . import _hip
from .model import LLaMA, _Work, _enable_i8_handoff


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
        if batch < 1:
            raise ValueError(f"decode batch {batch} < 1")
        # batches past QKV_ROWS (8) run every fused op in row slices of 8 (16 for the plain linears)
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
        if self.logits.dtype == torch.float32 and self.top_k != 1:  # the fp32 model: sampled in fp32
            _hip.call("llj_g_sample", self.logits.data_ptr(), self.logits.stride(0), self.B, cfg.padded_vocab_size,
                      self.temperature, self.top_k, _hip.ptr(self.uniforms), self.seed, self.cur.data_ptr(),
                      self.tokens.data_ptr(), self.total, self.pos.data_ptr(), st)
        elif self.logits.dtype == torch.float32:
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
            _enable_i8_handoff(self.work, self.specs)
        self.graph = None  # the caches / operands may have changed

    def _reset_handoff(self):
        """The LLM.int8 hand-off blocks (_Work.y_st / h_st) must be zero when a step starts; a
        completed step leaves them so, a step that raised part-way may not: zero them again."""
        w = self.work
        if w is not None and getattr(w, "y_st", None) is not None:
            w.y_st.zero_()
            w.h_st.zero_()

    def _step(self):
        try:
            self._step_launches()
        except BaseException:
            self._reset_handoff()
            raise

    def _step_launches(self):
        m, w, B = self.model, self.work, self.B
        cfg = m.config
        st = _hip.stream()
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
        return self.tokens[:, :self.t_prompt + self.steps_done]
