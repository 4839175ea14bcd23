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
+ MIOpen wgrad as above — or, when the conv's input is a fused BN+add+ReLU output
(every non-entry ResNet bottleneck), the data gradient is mivod's GEMM with that
BN's backward reduce in the epilogue (``_Conv1x1BN``, ``MIVOD_CONV_BN_BWD_FUSE``).
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


# Data-gradient filters of a whole model, made in ONE launch at the start of its training
# forward (``prepare_dgrad_filters``; csrc/kernels/mv_conv.hip transpose_filters_kernel)
# instead of a flip + layout copy / transpose copy per conv in backward (~55 launches per
# ResNet-50 step).  The map is live only inside that forward: an autograd function looks
# its filter up at FORWARD time and keeps it in ctx, so its backward uses exactly the
# filter of the weights it ran with.  (The buffers are reused by the next prepared
# forward: a graph kept across an optimizer step and a new forward would see the new
# weights' filters.)
_DGRAD_FILTERS: dict = {}


def prepare_dgrad_filters(convs) -> None:
    """Transposed, tap-rotated filters of ``convs`` (channels_last bf16 GPU Conv2d modules)
    in one launch; ``end_dgrad_filters()`` closes the window."""
    from . import kernels as K
    ws = [m.weight for m in convs]
    _DGRAD_FILTERS.clear()
    if not ws or os.environ.get("MIVOD_DGRAD_FILTERS", "1") == "0":
        return
    for w, wt in zip(ws, K.native().transpose_filters(ws)):
        _DGRAD_FILTERS[(w.data_ptr(), tuple(w.shape))] = wt


def end_dgrad_filters() -> None:
    _DGRAD_FILTERS.clear()


def dgrad_filter(w: torch.Tensor):
    """The prepared data-gradient filter of w ([C, K, k, k] channels_last) or None."""
    if not _DGRAD_FILTERS:
        return None
    return _DGRAD_FILTERS.get((w.data_ptr(), tuple(w.shape)))


def _wt_or_make(w: torch.Tensor, wt):
    return wt if wt is not None else _transposed_filter(w)


def dgrad1x1(dy: torch.Tensor, w: torch.Tensor, wt=None) -> torch.Tensor:
    """Input gradient of a stride-1 1x1 conv, dX = dY . W as an NHWC GEMM: mivod's
    256 x 256 kernel (mv_gemm256.hip) when Cin % 256 == 0 and Cout >= 256, mv_gemm's
    streaming kernel for Cout in {64, 128, 256} (ResNet-50 layer1.0's 64 -> 64 conv1: CK's
    forward solver + its output zero fill took 308 + 174 us at bs2048), else the forward
    conv with the transposed filter (CK)."""
    cout, cin = w.shape[0], w.shape[1]
    gemm_ok = (dy.is_cuda and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
               and dy.is_contiguous(memory_format=torch.channels_last) and cout % 64 == 0
               and cin % 64 == 0)
    # (wt: the prepared [cin, cout, 1, 1] channels_last transpose = W^T as [cin, cout])
    wt2 = wt.reshape(cin, cout) if wt is not None else w.reshape(cout, cin).t().contiguous()
    if gemm_ok and cin < 256 and cout in (64, 128, 256):
        from . import kernels as K
        n, _, h, wd = dy.shape
        m = n * h * wd
        dx = torch.empty(m, cin, dtype=dy.dtype, device=dy.device)
        K.native().gemm_nt(dy.permute(0, 2, 3, 1).reshape(m, cout), wt2, dx, None, None)
        return dx.view(n, h, wd, cin).permute(0, 3, 1, 2)
    if (gemm_ok and os.environ.get("MIVOD_GEMM256", "1") != "0" and cin % 256 == 0
            and cout >= 256):
        from . import kernels as K
        n, _, h, wd = dy.shape
        m = n * h * wd
        dx = torch.empty(m, cin, dtype=dy.dtype, device=dy.device)
        K.native().gemm_nt(dy.permute(0, 2, 3, 1).reshape(m, cout), wt2, dx, None, None)
        return dx.view(n, h, wd, cin).permute(0, 3, 1, 2)
    return F.conv2d(dy, _wt_or_make(w, wt))


def _wgrad1x1_on_mivod(cin: int, cout: int) -> bool:
    """mivod's 1x1 weight-gradient kernel (csrc/kernels/mv_conv.hip wgrad1x1_kernel) vs
    MIOpen's backward-weights solver on the ResNet-50 bs2048 shapes (scripts/
    micro_wgrad1x1.py, profiles/r2_wgrad1x1_vs_miopen.txt): level on the HBM-bound
    64-channel ones (kept on MIOpen), 3-23% faster from 128 channels up."""
    return (os.environ.get("MIVOD_WGRAD1X1", "1") != "0" and min(cin, cout) >= 128
            and cin % 64 == 0 and cout % 64 == 0)


def wgrad1x1(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int = 1) -> torch.Tensor:
    """dW of y = conv1x1(x, w, stride, pad 0) — mivod's kernel where it wins, else MIOpen."""
    if (_wgrad1x1_on_mivod(w.shape[1], w.shape[0]) and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last)
            and dy.is_contiguous(memory_format=torch.channels_last)):
        from . import kernels as K
        return K.native().wgrad1x1(x, dy, stride)
    _, dw, _ = torch.ops.aten.convolution_backward(
        dy, x, w, None, [stride, stride], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])
    return dw


class _ConvDgradFwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, pad):
        ctx.save_for_backward(x, w)
        ctx.pad = pad
        ctx.wt = dgrad_filter(w)
        return F.conv2d(x, w, None, 1, pad)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = (dgrad1x1(dy, w, ctx.wt) if w.shape[2] == 1 and w.shape[3] == 1
                  else F.conv2d(dy, _wt_or_make(w, ctx.wt), None, 1, ctx.pad))
        if ctx.needs_input_grad[1]:
            if w.shape[2] == 1 and w.shape[3] == 1:
                dw = wgrad1x1(dy, x, w)
            else:
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


class _Conv1x1BN(torch.autograd.Function):
    """1x1 stride-1 conv feeding a BatchNorm, with two optional fusions.

    Forward (``gemm``): y = conv1x1(x, w) via mv_gemm (NHWC GEMM) + [P, 2, Cout] BN
    statistics partials of y around ``shift`` (non-differentiable side output); else
    MIOpen's forward and an empty partial tensor.

    Backward (``slot``): when x is the output of a fused BN+add+ReLU (ops.bn, mode 3)
    whose shortcut gradient is already parked in its GradSlot, the data gradient runs
    as mv_gemm's streaming kernel with THAT BN's backward reduce in the epilogue:
    dz = mask ? dx + dy_shortcut : 0 is written instead of dx, the partials
    (sum dz, sum dz (x_bn - mean)) ride along, and both are handed to the BN through
    the slot (``slot.pending``) while autograd receives None for x.  The BN backward
    then skips its reduce pass (one full read of dx, dy2, x_bn and a write of dz).
    A shortcut gradient on a stride grid (stage-entry blocks, ops.bn.downsample_tap) is
    added on that grid inside the epilogue.
    """

    @staticmethod
    def forward(ctx, x, w, shift, gemm, slot):
        from . import kernels as K
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        if gemm:
            nat = K.native()
            m = n * h * wd
            a = x.permute(0, 2, 3, 1).reshape(m, cin)            # NHWC view, no copy
            b = w.permute(0, 2, 3, 1).reshape(cout, cin)
            yf = torch.empty(m, cout, dtype=x.dtype, device=x.device)
            part = torch.empty(nat.gemm_partials(m, cout, cin), 2, cout, dtype=torch.float32,
                               device=x.device)
            nat.gemm_nt(a, b, yf, shift, part)
            y = yf.view(n, h, wd, cout).permute(0, 3, 1, 2)
        else:
            y = F.conv2d(x, w)
            part = torch.empty(0, dtype=torch.float32, device=x.device)
        ctx.save_for_backward(x, w)
        ctx.slot = slot
        ctx.wt = dgrad_filter(w)
        ctx.mark_non_differentiable(part)
        # no zero-filled gradient for the statistics output (a fill kernel per call)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:                      # the output was not used
            return None, None, None, None, None
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            slot, ctx.slot = ctx.slot, None
            if (slot is not None and slot.bn is not None and slot.grad is not None
                    and slot.pending is None):
                from . import kernels as K
                n, cin, h, wd = x.shape
                cout, m = w.shape[0], n * h * wd
                xb, mask, vec = slot.bn
                dz = torch.empty_like(x)
                g2, s2 = slot.take_strided()      # stride > 1: a stage-entry shortcut's grid
                wt2 = (ctx.wt.reshape(cin, cout) if ctx.wt is not None
                       else w.reshape(cout, cin).t().contiguous())
                part = K.native().gemm_nt_bn_bwd(
                    dy.permute(0, 2, 3, 1).reshape(m, cout), wt2,
                    dz.permute(0, 2, 3, 1).reshape(m, cin), g2, mask,
                    None if slot.fold else xb.permute(0, 2, 3, 1).reshape(m, cin), vec, 0, s2,
                    h, wd)
                slot.pending = (dz, part)
            else:
                dx = dgrad1x1(dy, w, ctx.wt)
        if ctx.needs_input_grad[1]:
            dw = wgrad1x1(dy, x, w)
        return dx, dw, None, None, None


def stats_fusable(m: nn.Conv2d, x: torch.Tensor) -> bool:
    """1x1 / stride 1 convs whose forward mivod's GEMM runs at least as fast as
    MIOpen: K = Cin in {64, 128, 256} (the streaming kernel), Cin 512 -> Cout 128, and
    Cin >= 512 with Cout % 256 == 0 (the 256 x 256 kernel, mv_gemm256.hip:
    scripts/micro_gemm256.py, 1024 -> 256 at 14x14 bs2048 270 us vs CK 342 us)."""
    if os.environ.get("MIVOD_CONV_BN_FUSE", "1") == "0" or not _eligible(m, x):
        return False
    cin, cout = m.in_channels, m.out_channels
    big = (os.environ.get("MIVOD_GEMM256", "1") != "0" and cin >= 512 and cin % 64 == 0
           and cout % 256 == 0)
    return (tuple(m.kernel_size) == (1, 1) and cout % 64 == 0
            and (cin in (64, 128, 256) or (cin == 512 and cout == 128) or big))


def bwd_fusable(m: nn.Conv2d, x: torch.Tensor):
    """GradSlot of x's producer when this 1x1 conv's data gradient can carry that
    producer's BN backward reduce; else None.  Mode 3 (BN+add+ReLU, block input): the
    streaming GEMM with the bitmask/shortcut epilogue (Cout = the GEMM's K in {64, 128,
    256}).  (A mode-1 variant — conv3's data gradient as the implicit-GEMM kernel with
    ks = 1 carrying BN2's reduce — measured level on layer1 and 5-14% behind on layers 2-4
    (scripts/micro_dgrad_bn.py), bench A/B neutral, and was removed in round 3; the BN3
    fold computes conv3's data gradient itself.)"""
    slot = getattr(x, "_mv_slot", None)
    if (slot is None or getattr(slot, "bn", None) is None
            or os.environ.get("MIVOD_CONV_BN_BWD_FUSE", "1") == "0"
            or not (torch.is_grad_enabled() and x.requires_grad) or not _eligible(m, x)
            or tuple(m.kernel_size) != (1, 1) or m.in_channels % 64 != 0
            or m.out_channels % 64 != 0):
        return None
    mode = getattr(slot, "mode", 0)
    if mode == 3 and m.out_channels in (64, 128, 256):
        return slot
    return None


def conv1x1_bn(m: nn.Conv2d, x: torch.Tensor, shift, gemm: bool, slot):
    """(y, partial) — see _Conv1x1BN; ``shift`` is the BN's running mean (gemm only)."""
    return _Conv1x1BN.apply(x, m.weight, shift, gemm, slot)


def conv1x1_stats(m: nn.Conv2d, x: torch.Tensor, shift):
    """(y, partial) of the GEMM forward with fused statistics."""
    return _Conv1x1BN.apply(x, m.weight, shift, True, None)


# ---------------------------------------------------------------- 3x3 implicit GEMM
# scripts/micro_dgrad_bn.py (dgrad + BN1 backward, MIOpen vs mivod with the BN reduce in
# the epilogue): layer1 1858 -> 1654 us, layer2 1145 -> 1034 us, layer3 714 -> 743 us,
# layer4 633 -> 625 us; so mivod takes the <= 128-channel data gradients.  (Before the
# EPI-2 variant's register diet it ran one workgroup per CU and lost in the full step.)
_DGRAD_DEFAULT = "128"


def conv3x3_eligible(m: nn.Conv2d, x: torch.Tensor) -> bool:
    """3x3 / pad 1 / stride 1-2 convs on channels_last bf16 GPU tensors with channel
    counts that are multiples of 64 (every ResNet-50 bottleneck conv2)."""
    return (os.environ.get("MIVOD_CONV3X3", "1") != "0"
            and x.is_cuda and x.dtype == torch.bfloat16 and m.weight.dtype == torch.bfloat16
            and m.bias is None and m.groups == 1 and tuple(m.kernel_size) == (3, 3)
            and tuple(m.padding) == (1, 1) and tuple(m.dilation) == (1, 1)
            and m.stride[0] == m.stride[1] and m.stride[0] in (1, 2) and m.padding_mode == "zeros"
            and m.in_channels % 64 == 0 and m.out_channels % 64 == 0 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last))


def _dgrad_on_mivod(cin: int, cout: int) -> bool:
    """Whether the stride-1 data gradient (a forward 3x3 conv Cout -> Cin) runs on mivod's
    kernel — which also lets it carry the producing BN's backward reduce — instead of
    MIOpen's forward solver.  MIVOD_CONV3X3_DGRAD: 0 = never, 1 = always, N = up to N
    channels (default: see _DGRAD_DEFAULT, chosen by bench.py A/B)."""
    v = os.environ.get("MIVOD_CONV3X3_DGRAD", _DGRAD_DEFAULT)
    if v == "0":
        return False
    if v == "1":
        return True
    # the data gradient's output channels (cin) % 256 == 0: the 256 x 256 pipeline
    # (mv_gemm256.hip AMODE 3) — ahead of CK's forward solver on layers 3-4
    if cin % 256 == 0 and cin <= 2048 and os.environ.get("MIVOD_CONV256", "1") != "0":
        return True
    return max(cin, cout) <= int(v)


def _dgrad_s2_on_mivod(cin: int, h: int, w: int) -> bool:
    """Stride-2 data gradient as four output-parity-class gather GEMMs (mv_gemm256.hip AMODE
    4 for dx channels % 256 == 0, mv_conv.hip's conv3x3_kernel DG mode otherwise; even input
    H, W) instead of MIOpen's backward-data solver plus its zero fill (scripts/
    micro_dgrad_s2.py, bs2048: layer3 1087 -> 683 us, layer4 1038 -> 644 us).
    MIVOD_CONV3X3_DGRAD_S2=0 disables it."""
    return (os.environ.get("MIVOD_CONV3X3_DGRAD_S2", "1") != "0" and cin % 64 == 0
            and h % 2 == 0 and w % 2 == 0)



def _wgrad_on_mivod(cin: int, cout: int, stride: int) -> bool:
    """mivod's 3x3 weight-gradient kernel (csrc/kernels/mv_conv.hip wgrad3x3_kernel) beats
    MIOpen's on every ResNet-50 conv2 shape except the 512-channel stride-2 one
    (scripts/micro_conv3x3.py: 608-793 vs 393-743 TF/s)."""
    if os.environ.get("MIVOD_WGRAD3X3", "1") == "0":
        return False
    # C, K % 256 == 0: the 256 x 256 pipeline (mv_gemm256.hip wgrad256_kernel<9>), any stride
    if cin % 256 == 0 and cout % 256 == 0 and os.environ.get("MIVOD_WGRAD256_3X3", "1") != "0":
        return True
    return not (stride == 2 and max(cin, cout) >= 512)


class _Conv3x3(torch.autograd.Function):
    """y = conv3x3(x, w, stride, pad 1) on mivod's implicit-GEMM kernel (csrc/kernels/
    mv_conv.hip), optionally with the following BatchNorm's statistics partials of y
    around ``shift`` (non-differentiable second output).  Backward: stride-1 data
    gradient as a forward conv with the flipped, channel-transposed filter (mivod's
    kernel for <= 128 channels, MIOpen's forward solver otherwise) — and when x is the
    output of a fused BN+ReLU (``slot``, mode 1), mivod's kernel also runs that BN's
    backward reduce in its epilogue and hands (d, partials) to it through the slot, the
    same protocol as ``_Conv1x1BN``; the weight gradient on mivod's wgrad3x3 kernel
    (MIOpen for the 512-channel stride-2 conv); stride-2 data gradient on mv_gemm256's
    parity-class GEMMs (even input size), else MIOpen."""

    @staticmethod
    def forward(ctx, x, w, stride, shift, stats, slot):
        from . import kernels as K
        nat = K.native()
        wc = w.contiguous(memory_format=torch.channels_last)
        if stats:
            n, _, h, wd = x.shape
            ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
            k = w.shape[0]
            part = torch.empty(nat.conv3x3_partials(n * ho * wo, k), 2, k, dtype=torch.float32,
                               device=x.device)
            y = nat.conv3x3(x, wc, stride, shift, part)
        else:
            part = torch.empty(0, dtype=torch.float32, device=x.device)
            y = nat.conv3x3(x, wc, stride)
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        ctx.slot = slot
        ctx.wt = dgrad_filter(w)
        ctx.mark_non_differentiable(part)
        # no zero-filled gradient for the statistics output (a fill kernel per call)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:                      # the output was not used
            return None, None, None, None, None, None
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        s = ctx.stride
        slot, ctx.slot = ctx.slot, None
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if s == 1:
            if need_x:
                wt = _wt_or_make(w, ctx.wt)
                if _dgrad_on_mivod(w.shape[1], w.shape[0]):
                    from . import kernels as K
                    if (slot is not None and slot.bn is not None and slot.mode == 1
                            and slot.pending is None):
                        xb, _, vec = slot.bn
                        d, part = K.native().conv3x3_bn_bwd(dy, wt, xb, vec)
                        slot.pending = (d, part)
                    else:
                        dx = K.native().conv3x3(dy, wt, 1)
                else:
                    dx = F.conv2d(dy, wt, None, 1, 1)
        else:
            r = []
            if need_x and s == 2 and _dgrad_s2_on_mivod(w.shape[1], x.shape[2], x.shape[3]):
                from . import kernels as K
                r = K.native().conv3x3_s2_dgrad(dy, _wt_or_make(w, ctx.wt), x.shape[2],
                                                x.shape[3])
                if r:
                    dx = r[0]
            if need_x and not r:
                dx, _, _ = torch.ops.aten.convolution_backward(
                    dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])
        if need_w:
            if _wgrad_on_mivod(w.shape[1], w.shape[0], s):
                from . import kernels as K
                dw = K.native().wgrad3x3(x, dy, s)
            else:
                _, dw, _ = torch.ops.aten.convolution_backward(
                    dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])
        return dx, dw, None, None, None, None


def bwd3x3_fusable(m: nn.Conv2d, x: torch.Tensor):
    """GradSlot of x's producer when this 3x3 conv's data gradient runs on mivod's kernel
    (stride 1, or stride 2 on the parity-class GEMMs) and can carry that producer's
    BN+ReLU backward reduce; else None."""
    slot = getattr(x, "_mv_slot", None)
    if (slot is None or getattr(slot, "bn", None) is None or getattr(slot, "mode", 0) != 1
            or os.environ.get("MIVOD_CONV_BN_BWD_FUSE", "1") == "0"
            or os.environ.get("MIVOD_CONV3X3_BN_BWD", "1") == "0"
            or not (torch.is_grad_enabled() and x.requires_grad)):
        return None
    if m.stride[0] == 1 and _dgrad_on_mivod(m.in_channels, m.out_channels):
        return slot
    # (stride 2: a BN-reduce epilogue on the parity-class GEMMs measured slower than the
    # separate reduce pass — its scattered BN-input reads are latency-bound, 683 -> 1081 us
    # for the layer3 shape — so the producing BN keeps its own reduce there)
    return None


def conv3x3_bn(m: nn.Conv2d, x: torch.Tensor, shift, stats: bool, slot=None):
    """(y, partial) — see _Conv3x3; ``shift`` is the BN's running mean (stats only)."""
    return _Conv3x3.apply(x, m.weight, int(m.stride[0]), shift, stats, slot)


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict) with the forward-conv dgrad."""

    def forward(self, x):
        if _eligible(self, x):
            return _ConvDgradFwd.apply(x, self.weight, self.padding[0])
        return super().forward(x)
