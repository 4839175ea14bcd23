"""Conv2d whose data gradient runs as a FORWARD convolution.

For a stride-1 conv with "same" padding (1x1/pad 0, 3x3/pad 1) the input
gradient is itself a stride-1 convolution of dY with the channel-transposed,
180-degree-rotated filter:

    dX = conv2d(dY, W.transpose(0, 1).flip(2, 3), padding=k // 2)

On gfx950 MIOpen's forward path (CK ``grouped_conv_fwd`` XDL kernels) runs these
problems up to 2x faster than its backward-data solvers, which also zero-fill dX
first (``SubTensorOpWithScalar1d`` / ``fillBufferAligned``, 17-112 us each at
ResNet-50 bs512): in profiles/r1_resnet50_bs512_fused_stem_taps.md a layer3 3x3
conv runs forward in ~93 us but backward-data in ~190 us (~620 TFLOP/s) + a fill.
The weight gradient still comes from MIOpen's backward-weights solver
(``aten.convolution_backward`` with only the weight output requested).

Only stride-1, dilation-1, ungrouped convs with padding ``k // 2`` on channels_last
bf16 GPU tensors take this path; everything else is a plain ``nn.Conv2d``.
``MIVOD_CONV_DGRAD_FWD=0`` disables it (A/B switch).

``conv1x1_stats`` is the forward of a stride-1 1x1 conv as mivod's own MFMA GEMM
(csrc/kernels/mv_gemm.hip, weight-stationary streaming kernel for K <= 256) with
the FOLLOWING BatchNorm's statistics computed in the GEMM epilogue — the BN's
separate statistics pass over the conv output disappears.  Used only where the
GEMM is at least as fast as MIOpen's kernel (scripts/micro_gemm1x1.py,
profiles/r2_gemm1x1_fused_stats.md); its backward is the same forward-conv dgrad
+ MIOpen wgrad as above.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F


def _transposed_filter(w: torch.Tensor) -> torch.Tensor:
    wt = w.transpose(0, 1)
    if w.shape[2] > 1 or w.shape[3] > 1:
        wt = wt.flip(2, 3)
    return wt.contiguous(memory_format=torch.channels_last)


class _ConvDgradFwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, pad):
        ctx.save_for_backward(x, w)
        ctx.pad = pad
        return F.conv2d(x, w, None, 1, pad)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = F.conv2d(dy, _transposed_filter(w), None, 1, ctx.pad)
        if ctx.needs_input_grad[1]:
            _, dw, _ = torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [ctx.pad, ctx.pad], [1, 1], False, [0, 0], 1,
                [False, True, False])
        return dx, dw, None


def _eligible(m: nn.Conv2d, x: torch.Tensor) -> bool:
    k = m.kernel_size
    return (os.environ.get("MIVOD_CONV_DGRAD_FWD", "1") != "0"
            and x.is_cuda and x.dtype == torch.bfloat16 and m.weight.dtype == torch.bfloat16
            and m.bias is None and m.groups == 1 and tuple(m.stride) == (1, 1)
            and tuple(m.dilation) == (1, 1) and k[0] == k[1] and k[0] % 2 == 1
            and tuple(m.padding) == (k[0] // 2, k[1] // 2) and m.padding_mode == "zeros"
            and x.is_contiguous(memory_format=torch.channels_last))


class _Conv1x1Stats(torch.autograd.Function):
    """y = conv1x1(x, w) via mv_gemm (NHWC GEMM) + [P, 2, Cout] BN statistics
    partials of y around ``shift`` (non-differentiable side output)."""

    @staticmethod
    def forward(ctx, x, w, shift):
        from . import kernels as K
        nat = K.native()
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        m = n * h * wd
        a = x.permute(0, 2, 3, 1).reshape(m, cin)            # NHWC view, no copy
        b = w.permute(0, 2, 3, 1).reshape(cout, cin)
        yf = torch.empty(m, cout, dtype=x.dtype, device=x.device)
        part = torch.empty(nat.gemm_partials(m, cout, cin), 2, cout, dtype=torch.float32,
                           device=x.device)
        nat.gemm_nt(a, b, yf, shift, part)
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return yf.view(n, h, wd, cout).permute(0, 3, 1, 2), part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = F.conv2d(dy, _transposed_filter(w))
        if ctx.needs_input_grad[1]:
            _, dw, _ = torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])
        return dx, dw, None


def stats_fusable(m: nn.Conv2d, x: torch.Tensor) -> bool:
    """1x1 / stride 1 convs whose forward mivod's GEMM runs at least as fast as
    MIOpen (K = Cin in {64, 128, 256}, or Cin 512 -> Cout 128 on MI355X)."""
    if os.environ.get("MIVOD_CONV_BN_FUSE", "1") == "0" or not _eligible(m, x):
        return False
    cin, cout = m.in_channels, m.out_channels
    return (tuple(m.kernel_size) == (1, 1) and cout % 64 == 0
            and (cin in (64, 128, 256) or (cin == 512 and cout == 128)))


def conv1x1_stats(m: nn.Conv2d, x: torch.Tensor, shift):
    """(y, partial) — see _Conv1x1Stats; ``shift`` is the BN's running mean."""
    return _Conv1x1Stats.apply(x, m.weight, shift)


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict) with the forward-conv dgrad."""

    def forward(self, x):
        if _eligible(self, x):
            return _ConvDgradFwd.apply(x, self.weight, self.padding[0])
        return super().forward(x)
