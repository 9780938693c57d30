"""Quantized Linear replacements for the decode path, backed by the HIP library.

Drop-in for reference lit_llama/quantization.py:
  * ColBlockQuantizedLinear (338-421): same constructor, buffers and state_dict keys
    (`quant_weight` (N, K*bits/8) uint8 column-major, `scales`, `zeros`, `bias`); forward
    runs the gfx950 GEMV on the streaming tiling of the codes (bits=4: W4P, bits=8: W8P = two
    nibble planes in W4P tiles; csrc/w4pack.hip), into which `quant_weight` is repacked IN
    PLACE the first time the module runs (one copy of the weights on the device, ~3.3 GB at
    7B). state_dict(), get_weight() and .to()/.cuda() see the reference layout (unpacked on
    demand); any write to `quant_weight` (load_state_dict, pack_weight, in-place ops) is
    taken as a new reference-layout buffer and repacked on the next forward. The reference computes bits=8 (and
    any non-Triton case) as F.linear(inp, get_weight(inp.dtype)) (409-421), i.e. with weights
    rounded to bf16((q - z) * s); the kernel applies s to the exact integer sum instead
    (difference <= 1 bf16 ulp per weight, covered by the tests' tolerance).
  * Linear8bitLt (36-75): nn.Linear-compatible constructor; the weight is re-quantized to
    LLM.int8() row-wise int8 (CB, SCB) at construction and on load_state_dict; forward is
    the int8 MFMA GEMV with the fp16 outlier-column side product (threshold 6.0).
  * qlinear_4bit_weight (282-331): functional int4 linear on the reference buffers.
There is no CPU path: forward on a non-ROCm device raises.
"""
from __future__ import annotations

import math

import torch

from . import _hip

_DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
ROWS_PER_CALL = 16  # llj_linear handles M <= 16 rows per launch


def _linear_rows(wfmt: int, x2: torch.Tensor, W: torch.Tensor, sz, bias, out2: torch.Tensor, N: int, K: int):
    s = _hip.stream()
    M = x2.shape[0]
    for r0 in range(0, M, ROWS_PER_CALL):
        r = min(ROWS_PER_CALL, M - r0)
        _hip.call("llj_linear", wfmt, x2[r0].data_ptr(), x2.stride(0), W.data_ptr(), _hip.ptr(sz), _hip.ptr(bias),
                  out2[r0].data_ptr(), out2.stride(0), r, N, K, None, 0, None, s)


def _as_rows(inp: torch.Tensor, K: int) -> torch.Tensor:
    x2 = inp.reshape(-1, K)
    if x2.stride(-1) != 1 or x2.stride(0) % 8:
        x2 = x2.contiguous()
    return x2


# for correctness AND speed: the reference's class of the same name ("for correctness but
# with terrible perf") with its forward on the gfx950 int4 kernel
class ColBlockQuantizedLinear(torch.nn.Module):
    def __init__(self, in_features, out_features, bias: bool, *, bits, tile_cols):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.tile_cols = tile_cols if tile_cols != -1 else self.in_features
        self.bits = bits
        self.entries_per_byte = 8 // bits
        assert self.entries_per_byte > 0 and self.entries_per_byte * self.bits == 8
        assert in_features % self.entries_per_byte == 0
        self.register_buffer(
            "quant_weight",
            torch.empty((self.out_features, self.in_features // self.entries_per_byte), dtype=torch.uint8)
            .t().contiguous().t(),
        )
        self.register_buffer(
            "scales",
            torch.empty((self.out_features, (self.in_features + self.tile_cols - 1) // self.tile_cols)),
        )
        self.register_buffer("zeros", torch.empty_like(self.scales))
        assert isinstance(bias, bool)
        if bias:
            self.register_buffer("bias", torch.empty((self.out_features,)))
        else:
            self.register_buffer("bias", None)
        # derived device-side operand of the HIP kernel (not part of the state_dict)
        self.register_buffer("_sz", None, persistent=False)
        self._qkey = None   # (data_ptr, version) of quant_weight right after its in-place repack
        self._szkey = None  # (scales, zeros) identity the _sz pairs were built from
        self._g = None      # any-shape path: (key, fp32 scales, fp32 zeros)
        self._zint = None   # (_szkey, every zero an integer) -- zeros_integral()

    # ---- reference buffer utilities (quantization.py:374-409) -------------------------
    def pack_weight(self, weight):
        """reference quantization.py:374-388 (the GPTQ producer's packing)."""
        weight = weight.to(device=self.quant_weight.device, copy=True)
        for j in range(self.scales.size(1)):
            weight[:, j * self.tile_cols:(j + 1) * self.tile_cols] /= self.scales[:, j:j + 1]
            weight[:, j * self.tile_cols:(j + 1) * self.tile_cols] += self.zeros[:, j:j + 1]
        weight = weight.clamp_(min=0, max=2 ** self.bits - 1).to(dtype=torch.uint8)
        self.quant_weight.zero_()
        for nr in range(self.entries_per_byte):
            self.quant_weight += weight[:, nr::self.entries_per_byte] << (nr * self.bits)

    def get_weight(self, dtype=torch.float):
        """reference quantization.py:390-409: the dequantized (N, K) weight."""
        qw = self._reference_codes()
        weight = torch.empty((self.out_features, self.in_features), device=qw.device, dtype=dtype)
        mask = (1 << self.bits) - 1
        for nr in range(self.entries_per_byte):
            weight[:, nr::self.entries_per_byte] = ((qw >> (nr * self.bits)) & mask).float()
        for j in range(self.scales.size(1)):
            weight[:, j * self.tile_cols:(j + 1) * self.tile_cols] -= self.zeros[:, j:j + 1]
            weight[:, j * self.tile_cols:(j + 1) * self.tile_cols] *= self.scales[:, j:j + 1]
        return weight

    # ---- HIP path ---------------------------------------------------------------------
    def _groups(self) -> int:
        return self.scales.shape[1]

    def _supported(self) -> bool:
        if self.out_features % 16 or self.in_features % 128 or self.bits not in (4, 8):
            return False
        if self._groups() == 1:
            return True
        # grouped (tile_cols = g): int4 with every 128-deep k-chunk inside one group
        return self.bits == 4 and self.tile_cols % 128 == 0

    def _is_packed(self) -> bool:
        """quant_weight currently holds the streaming tiling (not the reference layout)."""
        qw = self.quant_weight
        return self._qkey is not None and self._qkey == (qw.data_ptr(), qw._version)

    def _reference_codes(self) -> torch.Tensor:
        """quant_weight in the reference layout: the buffer itself, or an unpacked copy."""
        qw = self.quant_weight
        if not self._is_packed():
            return qw
        N, K = self.out_features, self.in_features
        out = torch.empty((N, K // self.entries_per_byte), dtype=torch.uint8, device=qw.device).t().contiguous().t()
        _hip.call("llj_w4_unpack" if self.bits == 4 else "llj_w8_unpack", qw.data_ptr(), out.data_ptr(), N, K,
                  _hip.stream())
        return out

    def _prepare(self):
        """Repack quant_weight in place when it holds reference-layout codes (first run, or written
        since), and (re)build the fp32 (scale, offset + zero) pairs when scales / zeros changed."""
        qw, sc, zr = self.quant_weight, self.scales, self.zeros
        szkey = (sc.data_ptr(), sc._version, zr.data_ptr(), zr._version, qw.device)
        if self._is_packed() and szkey == self._szkey:
            return
        _hip.require_device(qw, "ColBlockQuantizedLinear.quant_weight")
        if not self._supported():
            raise NotImplementedError(
                f"ColBlockQuantizedLinear(bits={self.bits}, tile_cols={self.tile_cols}, groups={self._groups()}, "
                f"{self.in_features}->{self.out_features}) has no HIP kernel yet (supported: N % 16 == 0, "
                "K % 128 == 0; gptq.int4 / gptq.int8 with tile_cols=-1, int4 with tile_cols % 128 == 0)")
        N, K = self.out_features, self.in_features
        s = _hip.stream()
        if not self._is_packed():
            if not qw.t().is_contiguous():  # keep the reference's column-major storage
                self.quant_weight = qw = qw.t().contiguous().t()
            flat = qw.t().view(-1)  # physical (K*bits/8, N) row-major bytes
            tmp = torch.empty_like(flat)
            _hip.call("llj_w4_repack" if self.bits == 4 else "llj_w8_repack", flat.data_ptr(), tmp.data_ptr(), N, K,
                      s)
            flat.copy_(tmp)
            del tmp
            self._qkey = (qw.data_ptr(), qw._version)
        if szkey != self._szkey or self._sz is None or self._sz.device != qw.device:
            G = self._groups()
            if self._sz is None or self._sz.device != qw.device or self._sz.shape[0] != G * N:
                self._sz = torch.empty(G * N, 2, dtype=torch.float32, device=qw.device)
            # (scale, offset + zero) pairs; grouped: group-major (G, N), one row of pairs per group
            sc1, zr1 = sc.t().contiguous().reshape(G * N), zr.t().contiguous().reshape(G * N)
            if sc1.dtype not in _DTYPE_CODE or zr1.dtype != sc1.dtype:
                sc1, zr1 = sc1.float(), zr1.float()
            _hip.call("llj_w4_scale_zero" if self.bits == 4 else "llj_w8_scale_zero", sc1.data_ptr(), zr1.data_ptr(),
                      _DTYPE_CODE[sc1.dtype], self._sz.data_ptr(), G * N, s)
            self._szkey = szkey

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        if self._is_packed():  # the state dict carries the reference layout
            destination[prefix + "quant_weight"] = self._reference_codes()

    def _apply(self, fn, *args, **kwargs):
        # moving / casting the module: put the reference layout back first so the moved buffer
        # is what it claims to be (repacked again on its next forward)
        if self._is_packed():
            ref = self._reference_codes()
            self.quant_weight.t().view(-1).copy_(ref.t().reshape(-1))
            self._qkey = None
        self._szkey = None
        self._g = None
        self._zint = None
        return super()._apply(fn, *args, **kwargs)

    def zeros_integral(self) -> bool:
        """Every zero an integer of magnitude <= 240 (GPTQ's round(-min / scale), clamped to the code
        range): the prompt GEMMs then convert the codes into an exact bf16 (q - z) tile
        (LLJ_WF_ZINT, csrc/gemm.hip). One device sync per scales / zeros version; False while a
        graph is being captured (the default int4 kernel then runs)."""
        self._prepare()
        if self._zint is None or self._zint[0] != self._szkey:
            if torch.cuda.is_current_stream_capturing():
                return False
            zr = self.zeros.float()
            self._zint = (self._szkey, bool(torch.equal(zr, torch.round(zr))) and float(zr.abs().max()) <= 240.0)
        return self._zint[1]

    def _wspec(self):
        """(wfmt, weight operand, sz operand) for the fused model kernels."""
        self._prepare()
        return self.wfmt, self.quant_weight, self._sz

    def _gspec(self):
        """Operands of the any-shape kernel (llj_g_linear, csrc/generic.hip) for shapes the
        streaming tiling does not take: (0, quant_weight in the reference's column-major layout,
        fp32 scales (N, G), fp32 zeros (N, G), bits, group). Nothing is repacked."""
        qw = self._reference_codes()
        if qw is self.quant_weight and not qw.t().is_contiguous():
            self.quant_weight = qw = qw.t().contiguous().t()
        _hip.require_device(qw, "ColBlockQuantizedLinear.quant_weight")
        sc, zr = self.scales, self.zeros
        key = (sc.data_ptr(), sc._version, zr.data_ptr(), zr._version, qw.device)
        if self._g is None or self._g[0] != key:
            self._g = (key, sc.to(device=qw.device, dtype=torch.float32).contiguous(),
                       zr.to(device=qw.device, dtype=torch.float32).contiguous())
        return 0, qw, self._g[1], self._g[2], self.bits, self.tile_cols

    @property
    def wfmt(self) -> int:
        """C-ABI weight format: 0 = W4P (bits=4), 3 = W8P (bits=8), grouped int4 (tile_cols = g):
        4 (W4P tiles + per-group pairs) | (g / 128) << 8."""
        if self._groups() > 1:
            return 4 | ((self.tile_cols // 128) << 8)
        return 0 if self.bits == 4 else 3

    def forward(self, inp):
        _hip.require_device(inp, "input")
        if inp.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError(f"ColBlockQuantizedLinear HIP path computes in bfloat16 or float32, got {inp.dtype}")
        K, N = self.in_features, self.out_features
        if not self._supported() or inp.dtype == torch.float32:  # the any-shape kernel on the reference buffers
            if self.bias is not None:
                raise NotImplementedError("biased ColBlockQuantizedLinear on the any-shape / fp32 path")
            x2 = inp.reshape(-1, K).contiguous()
            out = torch.empty((x2.shape[0], N), dtype=inp.dtype, device=inp.device)
            kind, qw, sc, zr, bits, group = self._gspec()
            _hip.call("llj_g_linear", kind, x2.data_ptr(), K, x2.shape[0], K, qw.data_ptr(), sc.data_ptr(), zr.data_ptr(),
                      bits, group, N, out.data_ptr(), N, None, 0, 0 if inp.dtype == torch.bfloat16 else 1, _hip.stream())
            return out.reshape(*inp.shape[:-1], N)
        self._prepare()
        x2 = _as_rows(inp, K)
        out = torch.empty((x2.shape[0], N), dtype=inp.dtype, device=inp.device)
        bias = None if self.bias is None else self.bias.to(torch.bfloat16)
        _linear_rows(self.wfmt, x2, self.quant_weight, self._sz, bias, out, N, K)
        return out.reshape(*inp.shape[:-1], N)


def qlinear_4bit_weight(inp, weight, scales, zeros):
    """Functional form of reference quantization.py:282-331 on the reference buffers
    (`weight` = quant_weight (N, K/2), scales/zeros (N, 1))."""
    N, K = weight.shape[0], weight.shape[1] * 2
    lin = ColBlockQuantizedLinear(K, N, False, bits=4, tile_cols=-1).to(weight.device)
    lin.quant_weight = weight
    lin.scales = scales
    lin.zeros = zeros
    return lin(inp)


def int8_linear(x: torch.Tensor, CB: torch.Tensor, SCB: torch.Tensor, bias, threshold: float = 6.0):
    """LLM.int8() matmul of bf16 x (..., K) with the row-quantized (CB, SCB) weight; CB in the I8P
    tiling (Linear8bitLt keeps its weight that way, llj_i8_repack)."""
    K = x.shape[-1]
    N = CB.shape[0]
    x2 = _as_rows(x, K)
    M = x2.shape[0]
    s = _hip.stream()
    ws = torch.empty(_hip.lib().llj_i8_ws_bytes(M, K), dtype=torch.uint8, device=x.device)
    _hip.call("llj_i8_stats", x2.data_ptr(), x2.stride(0), M, K, threshold, ws.data_ptr(), s)
    out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    for r0 in range(0, M, 8):
        r = min(8, M - r0)
        _hip.call("llj_linear", 2, x2[r0].data_ptr(), x2.stride(0), CB.data_ptr(), SCB.data_ptr(), _hip.ptr(bias),
                  out[r0].data_ptr(), out.stride(0), r, N, K, ws.data_ptr(), r0, None, s)
    return out.reshape(*x.shape[:-1], N)


class Linear8bitLt(torch.nn.Module):
    """LLM.int8() Linear (reference quantization.py:36-75 over bnb.nn.Linear8bitLt with
    has_fp16_weights=False, threshold=6.0). `weight` holds the int8 row-quantized CB (N, K),
    `SCB` the fp32 row absmax (N,). Loading a float `weight` re-quantizes it."""

    threshold = 6.0

    def __init__(self, in_features, out_features, bias=True, device=None, dtype=None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self._ikey = None  # (data_ptr, version) of weight right after its in-place I8P tiling
        w = torch.empty((out_features, in_features), device=device, dtype=dtype)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = torch.nn.Parameter(w, requires_grad=False)
        self.register_buffer("SCB", None)
        if bias:
            self.bias = torch.nn.Parameter(torch.zeros(out_features, device=device, dtype=dtype), requires_grad=False)
        else:
            self.register_parameter("bias", None)
        # reference quantizes the initial weight right away (quantization.py:46-48); that
        # needs the GPU, exactly like the reference's `.cuda()` there
        if w.device.type == "cuda":
            self._quantize_weight(w)

    def _quantize_weight(self, weight: torch.Tensor) -> None:
        """double_quant(W.half()) equivalent: CB = round(W16 * 127 / absmax_row), SCB = absmax_row."""
        _hip.require_device(weight, "Linear8bitLt weight")
        w = weight.contiguous()
        if w.dtype not in _DTYPE_CODE:
            w = w.float()
        N, K = w.shape
        cb = torch.empty((N, K), dtype=torch.int8, device=w.device)
        scb = torch.empty((N,), dtype=torch.float32, device=w.device)
        _hip.call("llj_i8_quant_weight", w.data_ptr(), _DTYPE_CODE[w.dtype], cb.data_ptr(), scb.data_ptr(), N, K,
                  _hip.stream())
        self.weight = torch.nn.Parameter(cb, requires_grad=False)
        self.SCB = scb

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        key = prefix + "weight"
        if key in state_dict:
            w = state_dict[key]
            scb_key = prefix + "SCB"
            if w.dtype == torch.int8 and scb_key in state_dict:  # our own saved (CB, SCB) form
                self.weight = torch.nn.Parameter(w.to(self.weight.device).contiguous(), requires_grad=False)
                self.SCB = state_dict[scb_key].to(self.weight.device, torch.float32).contiguous()
            else:
                self._quantize_weight(w.to(self.weight.device))
        bkey = prefix + "bias"
        if self.bias is not None and bkey in state_dict:
            with torch.no_grad():
                self.bias.copy_(state_dict[bkey])
        for k in (key, prefix + "SCB", bkey):
            if k in missing_keys:
                missing_keys.remove(k)

    # ---- CB storage: the int8 GEMV reads the I8P tiling (llj_i8_repack: one contiguous KiB per
    # wave and MFMA step instead of 16 rows x 64 B), so `weight` is re-tiled IN PLACE the first
    # time it is used on the GPU; the state dict, `.to()` and `cb_reference()` see the row-major CB
    def _is_tiled(self) -> bool:
        w = self.weight
        return self._ikey is not None and self._ikey == (w.data_ptr(), w._version)

    def cb_reference(self) -> torch.Tensor:
        """CB (N, K) int8 row-major: the weight itself, or an un-tiled copy."""
        w = self.weight
        if not self._is_tiled():
            return w.detach()
        cb = torch.empty_like(w)
        _hip.call("llj_i8_unpack", w.data_ptr(), cb.data_ptr(), w.shape[0], w.shape[1], _hip.stream())
        return cb

    def _prepare(self):
        if self.SCB is None or self.weight.dtype != torch.int8:
            self._quantize_weight(self.weight)
        if self._is_tiled():
            return
        w = self.weight
        _hip.require_device(w, "Linear8bitLt weight")
        N, K = w.shape
        if N % 16 or K % 128:
            raise NotImplementedError(f"Linear8bitLt ({N}, {K}): the int8 kernels need N % 16 == 0 and K % 128 == 0")
        tiled = torch.empty_like(w)
        _hip.call("llj_i8_repack", w.data_ptr(), tiled.data_ptr(), N, K, _hip.stream())
        with torch.no_grad():
            w.copy_(tiled)
        self._ikey = (w.data_ptr(), w._version)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        if self._is_tiled():  # the state dict carries the row-major CB
            destination[prefix + "weight"] = self.cb_reference()

    def _apply(self, fn, *args, **kwargs):
        if self._is_tiled():  # moving / casting: put the row-major CB back first
            cb = self.cb_reference()
            with torch.no_grad():
                self.weight.copy_(cb)
            self._ikey = None
        return super()._apply(fn, *args, **kwargs)

    def zeros_integral(self) -> bool:
        """Every zero an integer of magnitude <= 240 (GPTQ's round(-min / scale), clamped to the code
        range): the prompt GEMMs then convert the codes into an exact bf16 (q - z) tile
        (LLJ_WF_ZINT, csrc/gemm.hip). One device sync per scales / zeros version; False while a
        graph is being captured (the default int4 kernel then runs)."""
        self._prepare()
        if self._zint is None or self._zint[0] != self._szkey:
            if torch.cuda.is_current_stream_capturing():
                return False
            zr = self.zeros.float()
            self._zint = (self._szkey, bool(torch.equal(zr, torch.round(zr))) and float(zr.abs().max()) <= 240.0)
        return self._zint[1]

    def _wspec(self):
        self._prepare()
        return 2, self.weight, self.SCB

    def _gspec(self):
        """Operands of the any-shape LLM.int8 kernel (llj_g_i8_linear) for K % 128 != 0: (2, CB
        row-major, SCB, None, 8, K)."""
        if self.SCB is None or self.weight.dtype != torch.int8:
            self._quantize_weight(self.weight)
        if self.bias is not None:
            raise NotImplementedError("biased Linear8bitLt outside the streaming tiling")
        return 2, self.cb_reference(), self.SCB, None, 8, self.in_features

    def forward(self, x):
        _hip.require_device(x, "input")
        if x.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError(f"Linear8bitLt HIP path computes on bfloat16 or float32 input, got {x.dtype}")
        # the any-shape LLM.int8 kernels: shapes outside the streaming tiling, and fp32 input (cast to
        # fp16 inside and the result back to fp32, as bitsandbytes' MatMul8bitLt does)
        if self.in_features % 128 or self.out_features % 16 or x.dtype == torch.float32:
            from .model import LLaMA

            K, N = self.in_features, self.out_features
            x2 = x.reshape(-1, K).contiguous()
            out = torch.empty((x2.shape[0], N), dtype=x.dtype, device=x.device)
            LLaMA._glinear(self._gspec(), x2, x2.shape[0], K, N, out, None, _hip.stream())
            return out.reshape(*x.shape[:-1], N)
        self._prepare()
        bias = None if self.bias is None else self.bias.to(torch.bfloat16)
        return int8_linear(x, self.weight, self.SCB, bias, self.threshold)


class GPTQQuantizer:
    """GPTQ producer (reference quantization.py:424-614; IST-DASLab GPTQ, arXiv:2210.17323):
    same constructor, `collect_input_stats` forward hook and `quantize() -> (ColBlockQuantizedLinear,
    error)`. The calibration Hessian, the Cholesky factors and the trailing block update are
    library work on the device (torch GEMM / rocSOLVER); the sequential 128-column loop and the
    ColBlock packing are the HIP kernels `llj_gptq_block` / `llj_colblock_pack` (csrc/gptq.hip).
    Supported: perchannel True / False and sym False / True (find_params_weight, reference 475-514),
    blocksize 16 / 32 / 64 / 128 (557; quantize/gptq.py uses the defaults: per-channel, asymmetric,
    128), groupsize -1 or a multiple of 128 (grouped scales: each group's (scale, zero) is found when
    the column loop reaches its first column, from the weights as updated so far (reference 571-577);
    with groupsize % 128 == 0 that is the start of a block), in_features % 128 == 0.
    fp32 weights reproduce the reference's op order;
    other weight dtypes are quantized from their fp32 value (the reference would round the
    packing step in that dtype). No CPU path."""

    def __init__(self, linear_module, *, bits, perchannel=True, sym=False, blocksize=128, percdamp=0.01,
                 groupsize=-1, actorder=False):
        assert isinstance(linear_module, torch.nn.Linear)
        if blocksize not in (16, 32, 64, 128) or (groupsize != -1 and (groupsize <= 0 or groupsize % 128)):
            raise NotImplementedError("GPTQQuantizer HIP path: blocksize 16 / 32 / 64 / 128, groupsize -1 or a "
                                      "multiple of 128")
        assert not (actorder and groupsize != -1), "The permutation trick does not work for grouped quantization"
        self.linear_module = linear_module
        self.dev = linear_module.weight.device
        self.rows, self.columns = linear_module.weight.shape
        if self.columns % 128:
            raise NotImplementedError(f"GPTQQuantizer HIP path needs in_features % 128 == 0, got {self.columns}")
        self.H = torch.zeros((self.columns, self.columns), device=self.dev)
        self.nsamples = 0
        self.bits = bits
        self.maxq = 2 ** bits - 1
        self.perchannel, self.sym, self.blocksize = perchannel, sym, blocksize
        self.percdamp, self.groupsize, self.actorder = percdamp, groupsize, actorder
        self.tile_cols = self.columns if groupsize == -1 else groupsize
        self.scales = torch.zeros((self.rows, (self.columns + self.tile_cols - 1) // self.tile_cols),
                                  dtype=linear_module.weight.dtype, device=self.dev)
        self.zeros = torch.zeros_like(self.scales)

    def find_params_weight(self, x):
        """reference 475-514. The row min / max reduce on the device (exact); the N-element divisions
        run on the host, because torch's device division by a scalar multiplies by its reciprocal
        (not the reference's correctly rounded quotient). perchannel=False: one (scale, zero) over
        the whole matrix, repeated per row (481-482, 503-506); sym: the range symmetric about 0 and
        zero = (maxq + 1) / 2 (488-492, 498-499)."""
        rows = x.shape[0]
        if not self.perchannel:
            x = x.flatten().unsqueeze(0)
        tmp = torch.zeros(x.shape[0], device=x.device)
        xmin = torch.minimum(x.min(1)[0], tmp).cpu()
        xmax = torch.maximum(x.max(1)[0], tmp).cpu()
        if self.sym:
            xmax = torch.maximum(torch.abs(xmin), xmax)
            neg = xmin < 0
            xmin[neg] = -xmax[neg]
        both0 = (xmin == 0) & (xmax == 0)
        xmin[both0] = -1
        xmax[both0] = +1
        scale = (xmax - xmin) / self.maxq
        zero = torch.full_like(scale, (self.maxq + 1) / 2) if self.sym else torch.round(-xmin / scale)
        if not self.perchannel:
            scale, zero = scale.repeat(rows), zero.repeat(rows)
        return scale.reshape(-1, 1).to(x.device), zero.reshape(-1, 1).to(x.device)

    def collect_input_stats(self, _1, inp, _2):
        """Forward hook, reference 516-530: running H = 2/n Σ x xᵀ (a device GEMM)."""
        inp = inp[0].detach()
        self.last_inp = inp
        if len(inp.shape) == 2:
            inp = inp.unsqueeze(0)
        tmp = inp.shape[0]
        if len(inp.shape) == 3:
            inp = inp.reshape((-1, inp.shape[-1]))
        inp = inp.t()
        self.H *= self.nsamples / (self.nsamples + tmp)
        self.nsamples += tmp
        inp = math.sqrt(2 / self.nsamples) * inp.float()
        self.H += inp.matmul(inp.t())

    def quantize(self):
        """reference 532-614 with the column loop on the GPU: returns (ColBlockQuantizedLinear, error)."""
        _hip.require_device(self.linear_module.weight, "GPTQQuantizer linear_module.weight")
        W = self.linear_module.weight.detach().to(dtype=torch.float, copy=True)
        scale, zero = self.find_params_weight(W)
        self.scales[:] = scale
        self.zeros[:] = zero
        H = self.H
        del self.H
        dead = torch.diag(H) == 0
        H[dead, dead] = 1
        W[:, dead] = 0
        perm = None
        if self.actorder:
            perm = torch.argsort(torch.diag(H), descending=True, stable=True)
            W = W[:, perm]
            H = H[perm][:, perm]
        damp = self.percdamp * torch.mean(torch.diag(H))
        diag = torch.arange(self.columns, device=self.dev)
        H[diag, diag] += damp
        H = torch.linalg.cholesky(H)
        H = torch.cholesky_inverse(H)
        Hinv = torch.linalg.cholesky(H, upper=True).contiguous()
        N, K, B = self.rows, self.columns, self.blocksize
        Wt = W.t().contiguous()  # (K, N): column i of all rows is one coalesced row
        Qt = torch.empty_like(Wt)
        Err = torch.empty((B, N), dtype=torch.float32, device=self.dev)
        loss = torch.zeros(N, dtype=torch.float32, device=self.dev)
        # the stored (scale, zero) -- rounded to the buffers' dtype, e.g. bf16 -- are what decode
        # dequantizes with, so the column loop's reconstructions and error feedback use them too
        # (fp32 buffers: the reference's values exactly)
        g = self.tile_cols
        G = self.scales.shape[1]
        s = _hip.stream()
        scg, zrg = [None] * G, [None] * G  # per group: the stored (scale, zero) as fp32 columns
        if G == 1:
            scg[0] = self.scales.reshape(-1).float().contiguous()
            zrg[0] = self.zeros.reshape(-1).float().contiguous()
        for i1 in range(0, K, B):
            i2 = i1 + B
            gi = i1 // g
            if G > 1 and i1 % g == 0:  # reference 571-577: the group's params from W as updated so far
                gs, gz = self.find_params_weight(Wt[i1:i1 + g].t())
                self.scales[:, gi] = gs.reshape(-1)
                self.zeros[:, gi] = gz.reshape(-1)
                scg[gi] = self.scales[:, gi].float().contiguous()
                zrg[gi] = self.zeros[:, gi].float().contiguous()
            _hip.call("llj_gptq_block_bs", Hinv.data_ptr(), K, i1, B, Wt.data_ptr(), N, scg[gi].data_ptr(),
                      zrg[gi].data_ptr(), self.bits, Qt.data_ptr(), Err.data_ptr(), loss.data_ptr(), s)
            if i2 < K:  # W[:, i2:] -= Err1 @ Hinv[i1:i2, i2:] (596), transposed
                Wt[i2:] -= Hinv[i1:i2, i2:].t().matmul(Err)
        if perm is not None:
            Qt = Qt[torch.argsort(perm)].contiguous()
        error = loss.sum().item() / 2
        q_module = ColBlockQuantizedLinear(self.linear_module.in_features, self.linear_module.out_features,
                                           self.linear_module.bias is not None, bits=self.bits,
                                           tile_cols=self.groupsize).to(self.dev)
        q_module.scales = self.scales
        q_module.zeros = self.zeros
        # pack_weight (374-388) into quant_weight's column-major storage ((K/epb, N) bytes)
        assert q_module.quant_weight.stride() == (1, N)
        epb = 8 // self.bits
        for gi in range(G):  # group gi's columns are the contiguous bytes [g0 / epb, g1 / epb) x N
            g0, g1 = gi * g, min(K, (gi + 1) * g)
            _hip.call("llj_colblock_pack", Qt[g0].data_ptr(), g1 - g0, N, scg[gi].data_ptr(), zrg[gi].data_ptr(),
                      self.bits, q_module.quant_weight.data_ptr() + (g0 // epb) * N, s)
        q_module.bias = self.linear_module.bias
        return q_module, error
