"""ResNet-50 (v1.5 topology, 25,557,032 parameters), written from scratch.

North-star workload (BASELINE.json configs 3/4): ResNet-50
bf16 on synthetic ImageNet.  MI355X choices: NHWC (``channels_last``) so
MIOpen / the conv kernels see the layout the matrix cores want, bf16 weights
and activations with BatchNorm affine params and running statistics kept in
fp32 (the mixed BN path; mivod's fused optimizer holds the fp32 master copy of
the bf16 weights).  No torchvision (not installed), no torch.compile / Triton.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import os

import torch.nn.functional as F

from ..ops.conv import (Conv2d, conv1x1_stats, end_dgrad_filters, prepare_dgrad_filters,
                        stats_fusable)
from ..ops import bn as _bn
from ..ops.bn import (BatchNorm2d, bn_relu_conv3x3, bn_relu_maxpool, conv_bn, downsample_tap,
                      global_avg_pool, pad_channels, shortcut_foldable, shortcut_fusable, tap)


def conv3x3(cin, cout, stride=1, groups=1, dilation=1):
    return Conv2d(cin, cout, 3, stride=stride, padding=dilation, groups=groups, bias=False,
                  dilation=dilation)


def conv1x1(cin, cout, stride=1):
    return Conv2d(cin, cout, 1, stride=stride, bias=False)


class _StemConvStats(torch.autograd.Function):
    """The stem conv on mivod's MFMA kernel (csrc/kernels/mv_stem.hip) with the following
    BN's statistics partials from its epilogue; weight gradient on mv_stem.hip's kernel too
    (MIVOD_STEM_WGRAD=0: MIOpen's solver; bench A/B 15,290/15,312 vs 15,278/15,240 img/s with
    the next row prefetched into registers — without the prefetch it was 0.8% behind)."""

    @staticmethod
    def forward(ctx, x4, w4, shift):
        # x4: the 3-channel image itself (the kernels read RGB pixels and stage them as 4
        # channels) or a zero-padded 4-channel one
        from ..ops import kernels as K
        z, part = K.native().stem_fwd(x4, w4, shift)
        ctx.save_for_backward(x4, w4)
        ctx.mark_non_differentiable(part)
        # no zero-filled gradient for the statistics output (a fill kernel per call)
        ctx.set_materialize_grads(False)
        return z, part

    @staticmethod
    def backward(ctx, dz, _dpart):
        x4, w4 = ctx.saved_tensors
        dw = None
        if ctx.needs_input_grad[1] and dz is not None:
            dz = dz.contiguous(memory_format=torch.channels_last)
            if os.environ.get("MIVOD_STEM_WGRAD", "1") != "0":
                from ..ops import kernels as K
                dw = K.native().stem_wgrad(x4, dz)
            else:
                dw = torch.ops.aten.convolution_backward(dz, pad_channels(x4, 4), w4, None, [2, 2],
                                                         [3, 3], [1, 1], False, [0, 0], 1,
                                                         [False, True, False])[1]
        return None, dw, None


class StemConv(nn.Conv2d):
    """The 7x7/2 stem conv.  Parameters stay [64, 3, 7, 7]; on the GPU path the
    3-channel NHWC image and the weight are zero-padded to 4 channels first
    (``MIVOD_STEM_CHANNELS``, default 4): MIOpen's gfx950 kernels for Cin=3 run
    the stem at ~170 TFLOP/s and need an extra 170 us zero-fill, Cin=4 is ~1.4x
    faster fwd+wgrad (scripts/micro_stem.py).  The zero channel contributes
    nothing, and its weight gradient is sliced away, so the math is unchanged."""

    def stem_kernel_ok(self, x) -> bool:
        """mivod's stem kernels apply: not MIVOD_STEM_KERNEL=0, a 224x224 bf16 channels_last
        GPU image, the ResNet stem geometry."""
        return not (os.environ.get("MIVOD_STEM_KERNEL", "1") == "0" or not x.is_cuda
                    or x.dtype != torch.bfloat16 or x.dim() != 4
                    or tuple(x.shape[1:]) != (3, 224, 224)
                    or not x.is_contiguous(memory_format=torch.channels_last)
                    or self.weight.dtype != torch.bfloat16
                    or tuple(self.weight.shape) != (64, 3, 7, 7)
                    or tuple(self.stride) != (2, 2) or tuple(self.padding) != (3, 3)
                    or self.bias is not None or self.groups != 1
                    or tuple(self.dilation) != (1, 1))

    def kernel_operands(self, x):
        """(image, 4-channel OHWC filter) as the stem kernels take them: the kernels read the
        3-channel image directly (MIVOD_STEM_PAD_INPUT=1: pad it first)."""
        w = F.pad(self.weight, (0, 0, 0, 0, 0, 1)).contiguous(memory_format=torch.channels_last)
        xin = pad_channels(x, 4) if os.environ.get("MIVOD_STEM_PAD_INPUT", "0") == "1" else x
        return xin, w

    def forward_stats(self, x, shift):
        """(conv(x), [P, 2, 64] BN statistics partials around ``shift``) on mivod's stem
        kernel, or None when it does not apply (see stem_kernel_ok)."""
        if not self.stem_kernel_ok(x):
            return None
        return _StemConvStats.apply(*self.kernel_operands(x), shift)

    def forward(self, x):
        cp = int(os.environ.get("MIVOD_STEM_CHANNELS", "4"))
        if (cp > x.shape[1] and x.is_cuda and x.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last)):
            c = x.shape[1]
            w = F.pad(self.weight, (0, 0, 0, 0, 0, cp - c)).contiguous(
                memory_format=torch.channels_last)
            return F.conv2d(pad_channels(x, cp), w, None, self.stride, self.padding)
        return super().forward(x)


class _StemBNReluMaxPool(torch.autograd.Function):
    """maxpool(relu(bn(stem_conv(x)))) with ONE backward pass over the stem rows: the
    pooled-level BN reduce (mv_pool.hip), then the stem weight-gradient kernel rebuilds each
    row's dz from the conv output and the pooled gradients while staging it
    (mv_stem.hip, MvStemPoolBwd) — the full-resolution dz (3.3 GB at bs 2048) is never
    written or read back.  Forward = _StemConvStats + ops.bn._BNReluMaxPool's kernels.
    The image gets no gradient (as in _StemConvStats)."""

    @staticmethod
    def forward(ctx, x4, w4, weight, bias, running_mean, running_var, momentum, eps, slot):
        from ..ops import kernels as K
        nat = K.native()
        z, part = nat.stem_fwd(x4, w4, running_mean)
        vec = nat.bn_finalize(part, weight, bias, running_mean, running_var, momentum, eps,
                              z.numel() // z.shape[1])
        y, idx = nat.maxpool_fwd(z, vec[2], vec[3], True, 3, 2, 1)
        ctx.save_for_backward(x4, z, vec, weight, idx, y)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        x4, z, vec, weight, idx, y = ctx.saved_tensors
        dw, dg, db = K.native().stem_wgrad_pool_bn(
            x4, dy.contiguous(memory_format=torch.channels_last), ctx.slot.take(), idx, y, z,
            vec, weight)
        return (None, dw if ctx.needs_input_grad[1] else None,
                dg if ctx.needs_input_grad[2] else None,
                db if ctx.needs_input_grad[3] else None, None, None, None, None, None)


def stem_bn_relu_maxpool(conv: "StemConv", bn: BatchNorm2d, pool: nn.MaxPool2d, x):
    """``pool(relu(bn(conv(x))))`` on _StemBNReluMaxPool, or None when it does not apply
    (MIVOD_STEM_POOL_FUSE=0, not training with running statistics, another pool window,
    an image that needs a gradient, the stem kernels off)."""
    if (os.environ.get("MIVOD_STEM_POOL_FUSE", "1") == "0" or not _bn._POOL_BN_BWD
            or os.environ.get("MIVOD_FUSED_BN", "1") == "0"
            or not (bn.training and bn.track_running_stats) or bn.weight is None
            or bn.bias is None or bn.weight.dtype != torch.float32
            or _bn._pool_args(pool) != (3, 2, 1) or x.requires_grad
            or not conv.stem_kernel_ok(x)):
        return None
    bn._mv_steps += 1
    momentum = bn.momentum
    if momentum is None:
        momentum = 1.0 / float(bn._mv_steps + int(bn.num_batches_tracked.item()))
    slot = _bn.GradSlot()
    y = _StemBNReluMaxPool.apply(*conv.kernel_operands(x), bn.weight, bn.bias, bn.running_mean,
                                 bn.running_var, float(momentum), float(bn.eps), slot)
    y._mv_slot = slot
    return y


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, zero_init_residual=False):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = BatchNorm2d(planes * self.expansion)
        self.downsample = downsample

    def forward(self, x):
        # conv_bn: a qualifying 1x1 conv computes its BN's statistics in the GEMM
        # epilogue (mivod.ops.conv), so the BN skips its statistics pass; conv1's data
        # gradient also runs the backward reduce of the BN that produced x
        r = bn_relu_conv3x3(self.conv1, self.bn1, self.conv2, self.bn2, x)
        if r is not None:
            # layer1: BN1 + ReLU applied inside conv2's row-patch kernels (never written)
            out = self.bn2(r[0], relu=True, stats=r[1], colsum=_bn._COLSUM)
        else:
            out = conv_bn(self.conv1, self.bn1, x, relu=True)
            # 3x3: mivod's implicit-GEMM conv with the BN statistics in its epilogue
            # (+ column sums of the BN2 output for conv3's folded weight gradient)
            out = conv_bn(self.conv2, self.bn2, out, relu=True, colsum=True)
        # the shortcut's gradient is added inside the backward of the op that
        # produced x (mivod.ops.bn.tap), not by a separate autograd add; a strided
        # 1x1 shortcut conv hands it over at its output resolution (downsample_tap).
        # The tap is recorded AFTER the main branch so that autograd (which runs the
        # most recently recorded ready node first) parks the shortcut gradient before
        # conv1's backward, which then finds it for the fused reduce.
        if self.downsample is None:
            identity = tap(x)
        else:
            conv, rest = self.downsample[0], self.downsample[1:]
            if len(rest) == 1 and shortcut_fusable(self.conv3, self.bn3, out, rest[0]):
                # the shortcut BN's apply runs inside conv3's recomputing GEMM epilogue: only
                # the shortcut conv's output (and its BN statistics) is materialised; with
                # the shortcut fold the shortcut conv + BN backward also join the block's
                # fused backward (x's gradient parked in its producer's slot)
                if shortcut_foldable(conv, x):
                    return conv_bn(self.conv3, self.bn3, out, relu=True, residual=x,
                                   res_bn=rest[0], res_conv=conv)
                if conv.stride[0] == 1 and stats_fusable(conv, x):
                    z, part = conv1x1_stats(conv, tap(x), rest[0].running_mean)
                elif rest[0].training and rest[0].track_running_stats:
                    # strided shortcut on the 256 x 256 GEMM with its BN's statistics
                    z, part = downsample_tap(x, conv, rest[0].running_mean)
                else:
                    z, part = downsample_tap(x, conv), None
                return conv_bn(self.conv3, self.bn3, out, relu=True, residual=z, res_bn=rest[0],
                               res_part=part)
            if conv.stride[0] == 1 and len(rest) == 1 and isinstance(rest[0], BatchNorm2d):
                identity = conv_bn(conv, rest[0], tap(x))
            else:
                identity = rest(downsample_tap(x, conv))
        # fused: relu(bn3(conv3(out)) + identity) in one pass (mivod.ops.bn)
        return conv_bn(self.conv3, self.bn3, out, relu=True, residual=identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = StemConv(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0], 1, zero_init_residual)
        self.layer2 = self._make_layer(128, layers[1], 2, zero_init_residual)
        self.layer3 = self._make_layer(256, layers[2], 2, zero_init_residual)
        self.layer4 = self._make_layer(512, layers[3], 2, zero_init_residual)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:          # after the generic init, which would undo it
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _make_layer(self, planes, blocks, stride, zir):
        down = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * Bottleneck.expansion, stride),
                                 BatchNorm2d(planes * Bottleneck.expansion))
        layers = [Bottleneck(self.inplanes, planes, stride, down, zir)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes, zero_init_residual=zir))
        return nn.Sequential(*layers)

    def _dgrad_convs(self):
        """The convs whose data-gradient filters backward uses (every Conv2d but the stem),
        when they are channels_last bf16 GPU filters; else []."""
        cv = getattr(self, "_mv_dgrad_convs", None)
        if cv is None:
            cv = [m for m in self.modules() if isinstance(m, nn.Conv2d)
                  and not isinstance(m, StemConv) and m.groups == 1]
            self._mv_dgrad_convs = cv
        ok = all(m.weight.is_cuda and m.weight.dtype == torch.bfloat16
                 and m.weight.is_contiguous(memory_format=torch.channels_last) for m in cv)
        return cv if ok else []

    def forward(self, x):
        prepared = False
        if self.training and torch.is_grad_enabled() and x.is_cuda:
            convs = self._dgrad_convs()
            if convs:
                # all data-gradient filters of this step in one launch (ops.conv)
                prepare_dgrad_filters(convs)
                prepared = True
        try:
            return self._forward(x)
        finally:
            if prepared:
                end_dgrad_filters()

    def _forward(self, x):
        r = None
        y = stem_bn_relu_maxpool(self.conv1, self.bn1, self.maxpool, x)
        if y is not None:
            x = self.layer4(self.layer3(self.layer2(self.layer1(y))))
            return self.fc(global_avg_pool(x))
        if self.bn1.training and self.bn1.track_running_stats:
            r = self.conv1.forward_stats(x, self.bn1.running_mean)
        if r is not None:       # stem conv with the BN statistics in its epilogue
            x = bn_relu_maxpool(r[0], self.bn1, self.maxpool, stats=r[1])
        else:
            x = bn_relu_maxpool(self.conv1(x), self.bn1, self.maxpool)   # fused stem
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(global_avg_pool(x))


def resnet50(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes, **kw)


def resnet101(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 4, 23, 3), num_classes, **kw)


def to_mixed_bf16(model: nn.Module, channels_last: bool = True) -> nn.Module:
    """bf16 conv/linear weights, fp32 BatchNorm (affine + running stats),
    channels_last memory format."""
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            m.to(torch.bfloat16)
    if channels_last:
        model.to(memory_format=torch.channels_last)
    return model
