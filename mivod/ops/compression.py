"""Gradient compression (parity: horovod/tensorflow/compression.py and
horovod/torch/compression.py).

``Compression.none`` / ``Compression.fp16`` keep Horovod's interface
(``compress(t) -> (t', ctx)``, ``decompress(t', ctx)``) for the generic named-op
path.  On the bucketed gradient path the cast never runs as a separate pass: the
compressor only names a *wire dtype*, and the hand-written pack kernel (K1/K4)
casts while packing, the fused optimizer (K6/K5) reads the compressed wire
buffer directly.  ``Compression.bf16`` is a mivod extension (same exponent range
as fp32, so no overflow risk for bf16/fp32 gradients).
"""
from __future__ import annotations

import torch


class Compressor:
    """Interface for compressing and decompressing a given tensor."""

    wire_dtype_map: dict = {}

    @staticmethod
    def compress(tensor):
        raise NotImplementedError

    @staticmethod
    def decompress(tensor, ctx):
        raise NotImplementedError

    @classmethod
    def wire_dtype(cls, dtype: torch.dtype) -> torch.dtype:
        return cls.wire_dtype_map.get(dtype, dtype)


class NoneCompressor(Compressor):
    """Default no-op compression."""

    @staticmethod
    def compress(tensor):
        return tensor, None

    @staticmethod
    def decompress(tensor, ctx):
        return tensor


class FP16Compressor(Compressor):
    """Compress floating point gradients to 16-bit IEEE half."""

    wire_dtype_map = {torch.float32: torch.float16, torch.float64: torch.float16,
                      torch.bfloat16: torch.float16}

    @staticmethod
    def compress(tensor):
        ctx = tensor.dtype
        if tensor.dtype.is_floating_point and tensor.dtype != torch.float16:
            tensor = _cast(tensor, torch.float16)
        return tensor, ctx

    @staticmethod
    def decompress(tensor, ctx):
        if ctx is not None and ctx.is_floating_point and tensor.dtype != ctx:
            tensor = _cast(tensor, ctx)
        return tensor


class BF16Compressor(Compressor):
    """Compress fp32 gradients to bfloat16 (mivod extension)."""

    wire_dtype_map = {torch.float32: torch.bfloat16, torch.float64: torch.bfloat16}

    @staticmethod
    def compress(tensor):
        ctx = tensor.dtype
        if tensor.dtype in (torch.float32, torch.float64):
            tensor = _cast(tensor, torch.bfloat16)
        return tensor, ctx

    @staticmethod
    def decompress(tensor, ctx):
        if ctx is not None and tensor.dtype != ctx:
            tensor = _cast(tensor, ctx)
        return tensor


def _cast(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.float16,
                                                        torch.bfloat16) and \
            dtype in (torch.float32, torch.float16, torch.bfloat16):
        from .kernels import flat_cast
        out = torch.empty(t.shape, dtype=dtype, device=t.device)
        flat_cast(t.view(-1), out.view(-1))
        return out
    return t.to(dtype)


class Compression:
    """Optional gradient compression algorithm used during allreduce."""

    none = NoneCompressor
    fp16 = FP16Compressor
    bf16 = BF16Compressor

    @staticmethod
    def by_name(name: str):
        return {"none": NoneCompressor, "": NoneCompressor, "fp16": FP16Compressor,
                "bf16": BF16Compressor}[name.lower()]
