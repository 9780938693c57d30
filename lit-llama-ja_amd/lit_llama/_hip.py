"""ctypes binding of the in-tree HIP library `_lljamd.so` (C ABI: include/lit_llama_amd.h).

The library is the only compute path of this package: there is no CPU or eager-PyTorch
fallback. If it is missing or the device is not a ROCm GPU, calls raise.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

# LLJ_LIB: another build of the same library (experiment variants built by _build.build(out=...,
# defines=...)); the product loads the in-tree _lljamd.so
LIB_PATH = Path(os.environ["LLJ_LIB"]) if os.environ.get("LLJ_LIB") else Path(__file__).resolve().parent / "_lljamd.so"

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float


# name -> argtypes (every function returns int: 0 ok, hipError_t, or 1000 = EINVAL)
SIGNATURES = {
    "llj_w4_repack": [_P, _P, _I, _I, _P],
    "llj_w4_unpack": [_P, _P, _I, _I, _P],
    "llj_w4_scale_zero": [_P, _P, _I, _P, _I, _P],
    "llj_w8_repack": [_P, _P, _I, _I, _P],
    "llj_w8_unpack": [_P, _P, _I, _I, _P],
    "llj_i8_repack": [_P, _P, _I, _I, _P],
    "llj_i8_unpack": [_P, _P, _I, _I, _P],
    "llj_w8_scale_zero": [_P, _P, _I, _P, _I, _P],
    "llj_linear": [_I, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P],
    "llj_norm_qkv_rope": [_I, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I,
                          _P],
    "llj_attention_split": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P],
    "llj_gemm_i8_linear": [_P, _I, _P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P],
    "llj_gemm_i8_resid": [_P, _I, _P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P],
    "llj_gemm_i8_silu_mul": [_P, _I, _P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P],
    "llj_gemm_i8_qkv_rope": [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "llj_i8_gather_act": [_P, _I, _I, _I, _P, _P, _I, _P],
    "llj_i8_gather_weight": [_P, _P, _I, _I, _P, _P, _I, _P],
    "llj_gptq_block": [_P, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P],
    "llj_gptq_block_bs": [_P, _I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P],
    "llj_colblock_pack": [_P, _I, _I, _P, _P, _I, _P, _P],
    "llj_attention": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "llj_attention_prefill": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "llj_linear_resid": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P],
    "llj_linear_resid_attn": [_I, _P, _I, _I, _P, _P, _P, _I, _I, _I, _P, _P],
    "llj_attention_part": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P],
    "llj_norm_swiglu": [_I, _P, _P, _F, _P, _P, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _I, _P],
    "llj_norm_linear": [_I, _P, _P, _F, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P],
    "llj_i8_stats": [_P, _I, _I, _I, _F, _P, _P],
    "llj_i8_norm_stats": [_P, _P, _F, _P, _I, _I, _F, _P, _P],
    "llj_i8_quant_weight": [_P, _I, _P, _P, _I, _I, _P],
    "llj_embedding": [_P, _P, _P, _I, _I, _P, _P],
    "llj_rmsnorm": [_P, _P, _F, _P, _I, _I, _P],
    "llj_rmsnorm_rows": [_P, _P, _F, _P, _P, _I, _I, _P],
    "llj_argmax": [_P, _I, _I, _I, _P, _P, _I, _P, _P],
    "llj_sample": [_P, _I, _I, _I, _F, _I, _P, ctypes.c_ulonglong, _P, _P, _I, _P, _P],
    "llj_set_tpw_max": [_I],
    "llj_set_stream_a": [_I],
    "llj_set_option": [_I, _I],
    "llj_attention_i8": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P],
    "llj_i8_swiglu_stats": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _F, _P],
    "llj_i8_norm_rowstats": [_P, _P, _F, _P, _I, _I, _F, _P, _P, _P],
    "llj_i8_linear_resid": [_P, _I, _P, _P, _P, _I, _I, _I, _I, _P, _P],
    "llj_gemm_linear": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P],
    "llj_gemm_resid": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P],
    "llj_gemm_silu_mul": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P],
    "llj_gemm_swiglu": [_I, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P],
    "llj_gemm_swiglu_ws": [_I, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, ctypes.c_size_t, _P],
    "llj_gemm_resid_ws": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _P, ctypes.c_size_t, _P],
    "llj_gemm_qkv_rope": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "llj_stream_read": [_P, ctypes.c_size_t, _P, _I, _P],
    "llj_g_embedding": [_P, _P, _P, _I, _I, _P, _I, _P],
    "llj_g_rmsnorm": [_P, _I, _P, _F, _P, _I, _I, _I, _I, _P],
    "llj_g_linear": [_I, _P, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _I, _I, _P],
    "llj_g_rope_kv": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "llj_g_attention": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "llj_g_silu_mul": [_P, _P, _P, ctypes.c_size_t, _I, _P],
    "llj_g_argmax": [_P, _I, _I, _I, _P, _P, _I, _P, _P],
    "llj_g_sample": [_P, _I, _I, _I, _F, _I, _P, ctypes.c_ulonglong, _P, _P, _I, _P, _P],
    "llj_g_i8_linear": [_P, _I, _I, _I, _P, _P, _F, _P, _I, _P, _I, _P, _I, _I, _P],
}

_lib = None


class HipError(RuntimeError):
    pass


# llj_set_option indices (include/lit_llama_amd.h LLJ_OPT_*)
WF_I8_ROWSTATS = 0x10000  # wfmt flag: i8ws is a decode hand-off block (include/lit_llama_amd.h)
WF_ZINT = 0x20000  # prefill GEMM wfmt flag: int4 whose zeros are all integers (include/lit_llama_amd.h)
(OPT_ATT_SPEC_FULL, OPT_FLASH_QB, OPT_FLASH_PAIR, OPT_GEMM_GLDS, OPT_GLDS_COST128, OPT_GEMV_LDS_A_KB,
 OPT_ATT_SPEC_BATCH, OPT_GEMM_W4Z) = range(8)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise HipError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no fallback path.")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, argt in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = argt
            f.restype = ctypes.c_int
        L.llj_i8_ws_bytes.argtypes = [_I, _I]
        L.llj_i8_ws_bytes.restype = ctypes.c_size_t
        L.llj_attention_ws_bytes.argtypes = [_I, _I, _I, _I]
        L.llj_attention_ws_bytes.restype = ctypes.c_size_t
        L.llj_g_i8_ws_bytes.argtypes = [_I, _I]
        L.llj_g_i8_ws_bytes.restype = ctypes.c_size_t
        L.llj_i8_rowstats_bytes.argtypes = [_I]
        L.llj_i8_rowstats_bytes.restype = ctypes.c_size_t
        L.llj_gemm_resid_ws_bytes.argtypes = [_I, _I, _I, _I]
        L.llj_gemm_resid_ws_bytes.restype = ctypes.c_size_t
        L.llj_gemm_swiglu_ws_bytes.argtypes = [_I, _I, _I, _I]
        L.llj_gemm_swiglu_ws_bytes.restype = ctypes.c_size_t
        _lib = L
    return _lib


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        what = "unsupported shape/argument (EINVAL)" if rc == 1000 else f"hipError {rc}"
        raise HipError(f"{name} failed: {what}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def require_device(t: torch.Tensor, what: str = "tensor") -> None:
    if t.device.type != "cuda" or torch.version.hip is None:
        raise HipError(
            f"{what} is on {t.device}: this package runs only on a ROCm GPU (MI355X / gfx950); "
            "it has no CPU path")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
