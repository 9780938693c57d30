"""Plumbing for the quantized decode path: the Linear-substitution context managers and the
small helpers the model needs. Mirrors reference lit_llama/utils.py (same names, argument
meaning and error behaviour); the training/FSDP/DeepSpeed checkpoint helpers of that file
are out of scope.
"""
from __future__ import annotations

import functools
from contextlib import contextmanager

import torch
import torch.utils._device

from .checkpoint import incremental_save, lazy_load  # noqa: F401  (reference utils.py:364-376, 492-531)

llama_model_sizes = {  # reference utils.py:19-27
    512: "19M",
    640: "49M",
    780: "125M",
    4096: "7B",
    5120: "13B",
    6656: "30B",
    8192: "65B",
}


def llama_model_lookup(checkpoint: dict) -> str:
    """reference utils.py:30-36: model name from the embedding width."""
    embedding_size = checkpoint["transformer.wte.weight"].shape[1]
    return llama_model_sizes[embedding_size]


def find_multiple(n: int, k: int) -> int:
    """reference utils.py:39-42"""
    if n % k == 0:
        return n
    return n + k - (n % k)


def _quantized_linear_cls(mode):
    if mode == "llm.int8":
        from .quantization import Linear8bitLt

        return Linear8bitLt
    if mode == "gptq.int4":
        from .quantization import ColBlockQuantizedLinear

        return functools.partial(ColBlockQuantizedLinear, bits=4, tile_cols=-1)
    if mode == "gptq.int8":
        from .quantization import ColBlockQuantizedLinear

        return functools.partial(ColBlockQuantizedLinear, bits=8, tile_cols=-1)
    return None


class EmptyInitOnDevice(torch.overrides.TorchFunctionMode):
    """reference utils.py:105-170: build modules directly on `device`/`dtype`, skip
    torch.nn.init, and substitute torch.nn.Linear by the quantized class of `quantization_mode`."""

    def __init__(self, device=None, dtype=None, quantization_mode=None):
        self.quantization_mode = quantization_mode
        self.quantized_linear_cls = None
        if quantization_mode == "llm.int8":
            if device is None or torch.device(device).type != "cuda":
                raise ValueError("Quantization is only supported on the GPU.")
        if quantization_mode is not None:
            self.quantized_linear_cls = _quantized_linear_cls(quantization_mode)
            if self.quantized_linear_cls is None:
                raise RuntimeError(f"unknown quantization mode {quantization_mode}")
        self.device = None if device is None else torch.device(device)
        self.dtype = dtype

    def __enter__(self):
        if self.quantized_linear_cls is not None:
            self.torch_linear_cls = torch.nn.Linear
            torch.nn.Linear = self.quantized_linear_cls
        return super().__enter__()

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self.quantized_linear_cls is not None:
            torch.nn.Linear = self.torch_linear_cls
        return super().__exit__(exc_type, exc_val, exc_tb)

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if getattr(func, "__module__", None) == "torch.nn.init":
            if "tensor" in kwargs:
                return kwargs["tensor"]
            return args[0]
        ctors = torch.utils._device._device_constructors()
        if self.device is not None and func in ctors and kwargs.get("device") is None:
            kwargs["device"] = self.device
        if self.dtype is not None and func in ctors and kwargs.get("dtype") is None:
            kwargs["dtype"] = self.dtype
        return func(*args, **kwargs)


@contextmanager
def quantization(mode: str = None):
    """reference utils.py:173-194: while active, `torch.nn.Linear` is the quantized class of
    `mode` ('llm.int8' -> Linear8bitLt, 'gptq.int4' / 'gptq.int8' -> ColBlockQuantizedLinear
    with one (scale, zero) per output row). Unknown modes raise ValueError. Unlike the
    reference, the original class is restored even if the body raises."""
    quantized_linear_cls = None
    if mode is not None:
        quantized_linear_cls = _quantized_linear_cls(mode)
        if quantized_linear_cls is None:
            raise ValueError(f"Unknown quantization mode: {mode}")
    torch_linear_cls = torch.nn.Linear
    if quantized_linear_cls is not None:
        torch.nn.Linear = quantized_linear_cls
    try:
        yield
    finally:
        torch.nn.Linear = torch_linear_cls
