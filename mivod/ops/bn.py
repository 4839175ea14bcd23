"""Fused BatchNorm2d (+ residual add) (+ ReLU) for channels_last bf16 activations.

``BatchNorm2d`` is a drop-in subclass of ``torch.nn.BatchNorm2d`` (same
parameters, buffers and state_dict) whose ``forward(x, residual=None,
relu=False)`` computes ``act(bn(x) + residual)`` in one fused pass with the
hand-written gfx950 kernels of ``csrc/kernels/mv_bn.hip`` (fp32 statistics and
affine params, bf16 activations).  Any other input (CPU, fp32, NCHW, C % 8 != 0)
takes the plain PyTorch path with identical semantics.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K

# MIVOD_BN_MASK=0: add+ReLU backward re-reads the bf16 output (mode 2) instead of the
# forward's bitmask (mode 3) -- A/B switch
_BN_MASK = os.environ.get("MIVOD_BN_MASK", "1") != "0"
# MIVOD_BN_RECOMPUTE=0: the BN3 fold materialises z and runs the separate apply pass (A/B)
_RECOMPUTE = os.environ.get("MIVOD_BN_RECOMPUTE", "1") != "0"
# ... for K = Cin <= MIVOD_BN_RECOMPUTE_MAXK (default 256; blocks with a projection shortcut
# always, their BN is applied in that epilogue).  With a statistics-only GEMM pass, K = 256
# (ResNet-50 layer3) was level (round 2: 15,294 / 15,330 vs 15,304 / 15,282 img/s at 128 vs
# 256); with the Gram statistics (_gram_stats) and 32-row apply tiles it wins (round 3 A/B:
# 17,441 vs 17,283 img/s)
_RECOMPUTE_MAXK = int(os.environ.get("MIVOD_BN_RECOMPUTE_MAXK", "256"))
# the 256 x 256 GEMM (mv_gemm256.hip) for the strided shortcut forward
_GEMM256 = os.environ.get("MIVOD_GEMM256", "1") != "0"
# MIVOD_BN_FOLD_DX=0: the fold's data gradient runs as two hipBLASLt GEMMs and BN2 runs its
# own backward reduce pass, instead of mv_gemm's dual-source kernel with that reduce fused
_FOLD_DX = os.environ.get("MIVOD_BN_FOLD_DX", "1") != "0"
# MIVOD_BN_SHORTCUT=0: a projection shortcut's BN writes its output (identity) in its own
# apply pass instead of being applied inside the recomputing conv3 GEMM's epilogue
_SHORTCUT = os.environ.get("MIVOD_BN_SHORTCUT", "1") != "0"
# MIVOD_BN_SHORTCUT_FOLD=0: the projection shortcut conv + BN keep their own backward (BN
# reduce + dx passes, then the conv's data / weight gradients) instead of folding into
# the block's fused backward
_SHORTCUT_FOLD = os.environ.get("MIVOD_BN_SHORTCUT_FOLD", "1") != "0"
# MIVOD_BN_COLSUM=0: the fold's colsum(x) term reads x in a statistics pass instead of
# taking BN2's apply-pass column sums
_COLSUM = os.environ.get("MIVOD_BN_COLSUM", "1") != "0"
# MIVOD_BN_STATS_GRAM=0: the recomputed expansion conv's BN statistics come from a
# statistics-only GEMM pass over z = x W^T instead of x's Gram matrix (_gram_stats)
_GRAM_STATS = os.environ.get("MIVOD_BN_STATS_GRAM", "1") != "0"
# MIVOD_BN_SHORTCUT_DUAL=0: a stride-1 shortcut conv's output is written by its statistics
# GEMM and read back as the residual, instead of being recomputed inside conv3's apply GEMM
_SHORTCUT_DUAL = os.environ.get("MIVOD_BN_SHORTCUT_DUAL", "1") != "0"
# MIVOD_BN_FOLD_MATH=0: the fold's per-channel coefficients and small products run as
# eager PyTorch ops (~22 kernels per block) instead of mv_fold.hip's two kernels
_FOLD_MATH = os.environ.get("MIVOD_BN_FOLD_MATH", "1") != "0"
# MIVOD_POOL_BN_BWD=0: the stem's maxpool backward writes the pool-input gradient and the
# BN+ReLU backward runs its own reduce and dx passes over it
_POOL_BN_BWD = os.environ.get("MIVOD_POOL_BN_BWD", "1") != "0"
# MIVOD_BN_DUAL_WGRAD=0: the fold's dz^T x and Gram x^T x as two wgrad1x1 launches
_DUAL_WGRAD = os.environ.get("MIVOD_BN_DUAL_WGRAD", "1") != "0"


def _gram_stats(nat, x, w2, colsum, shift, m):
    """[1, 2, cout] statistics partials of z = x W^T around ``shift`` without computing z:
    sum z = W colsum(x) and sum z^2 = rowsum((W G) * W) with G = x^T x (mivod's wgrad1x1
    kernel, fp32) — one pass over x at 2 m cin^2 flops instead of the GEMM's 2 m cin cout,
    and colsum(x) comes for free from the producing BN's apply (``colsum`` [P, cin]); the
    [cout]-sized remainder is one kernel (mv_fold.hip gram_stats_kernel).
    Sums of the fp32 products: z itself is later rounded to bf16 (a ~2^-9 relative
    difference per element that the statistics average out)."""
    g = nat.wgrad1x1(x, x, 1, True)
    return nat.gram_stats(w2.contiguous(), g, colsum.sum(0), shift, m)


def _fold_math(nat, wb, g, gram, vec, gamma, m, part, sdz, colsum, xs_fn, need_w):
    """The BN fold's small-matrix math: (dgamma, dbeta, dW bf16 [cout, cin] or None,
    bcat bf16 [cin, cout + cin], badd fp32 [cin]) with dx = [dz | x] . bcat^T + badd.
    ``wb`` = W [cout, cin] bf16, ``g`` = dz^T x, ``gram`` = x^T x (need_w), ``part`` =
    the consumer's reduce partials (sum dz; or ``sdz`` given), ``colsum`` = [P, cin]
    column-sum partials of x or None (then ``xs_fn()`` gives colsum(x))."""
    cout, cin = g.shape
    if _FOLD_MATH and part is not None and cout % 64 == 0 and cin % 64 == 0:
        co, xsum = nat.fold_coeffs(part, wb, g, vec, gamma, m, colsum)
        if need_w and colsum is None:
            xsum = xs_fn().contiguous()
        dw, bcat, badd = nat.fold_products(wb, g, gram, co, xsum, need_w)
        return co[0], co[1], (dw if need_w else None), bcat, badd
    w2 = wb.float()
    if sdz is None:
        sdz = part[:, 0].sum(0)
    # sum dz (z - mean) = rowdot(W, G) - mean * sum dz, with z = x W^T
    sdzx = (w2 * g).sum(1) - vec[0] * sdz
    co = nat.bn_bwd_coeffs(vec, gamma, torch.stack((sdz, sdzx)).unsqueeze(0), m)
    ca, cb, cc = co[2], co[3], co[4]
    dw = None
    if need_w:
        xs = colsum.sum(0) if colsum is not None else xs_fn()
        dwf = torch.addcmul(ca[:, None] * g, cb[:, None], w2 @ gram)
        dwf.addr_(cc, xs)
        dw = dwf.to(wb.dtype)
    bcat = torch.cat(((ca[:, None] * w2).t(), w2.t() @ (cb[:, None] * w2)), 1).to(
        wb.dtype).contiguous()
    return co[0], co[1], dw, bcat, (cc @ w2).contiguous()


def _fusable(x: torch.Tensor, weight) -> bool:
    if os.environ.get("MIVOD_FUSED_BN", "1") == "0":     # eager reference path (tests)
        return False
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.size(1) % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and (weight is None or weight.dtype == torch.float32))


def _cl(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


class GradSlot:
    """Side channel for a second gradient stream of a fused op's output.

    A residual network uses a block's input twice (main branch + shortcut);
    autograd would sum the two gradients with a separate elementwise kernel
    (3 HBM passes of the activation).  Instead the shortcut use goes through
    ``tap(x)``, whose backward parks its gradient here and returns None, and
    the op that PRODUCED x reads it as ``dy2`` inside its own backward kernel
    (1 extra read).  Autograd still orders the producer after the tap: a None
    gradient satisfies the dependency edge.
    """
    __slots__ = ("grad", "stride", "full_shape", "bn", "mode", "pending", "fold", "colsum")

    def __init__(self):
        self.grad = None
        self.stride = 1          # > 1: grad is on the stride-s grid (downsample_tap)
        self.full_shape = None   # the tapped output's shape when stride > 1
        # (x, mask, vec) of the producing BN (mode 3: add+ReLU with its bitmask; mode 1:
        # ReLU, mask None), for a consumer conv whose data-gradient kernel runs this BN's
        # backward reduce (ops.conv._Conv1x1BN / _Conv3x3) ...
        self.bn = None
        self.mode = 0
        # ... and its result (dz, partials), consumed by the BN backward
        self.pending = None
        # producer is _Conv1x1BNFold: the consumer's reduce only needs sum dz (the
        # producer derives sum dz (x - mean) from its weight-gradient GEMM)
        self.fold = False
        # [P, C] column-sum partials of the output (BN+ReLU forward with colsum=True), for
        # a folded consumer's dW term cc (x) colsum(x)
        self.colsum = None

    def take(self):
        g, self.grad = self.grad, None
        if g is not None and self.stride > 1:      # a consumer without strided support
            s, self.stride = self.stride, 1
            full = torch.zeros(self.full_shape, dtype=g.dtype, device=g.device).contiguous(
                memory_format=torch.channels_last)
            full[:, :, ::s, ::s] = g
            return full
        return g

    def take_strided(self):
        """(grad, stride) for kernels that read a stride-grid gradient directly."""
        g, s = self.grad, self.stride
        self.grad, self.stride = None, 1
        return g, s


class _Tap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g.dim() == 4:
            g = g.contiguous(memory_format=torch.channels_last)
        assert ctx.slot.stride == 1, "a tapped output has one shortcut consumer"
        ctx.slot.grad = g if ctx.slot.grad is None else ctx.slot.grad + g
        return None, None


class _DownsampleTapConv(torch.autograd.Function):
    """Shortcut ``conv1x1(x, stride=s)`` of a tapped output (ResNet stage entry).
    Backward: dW from ops.conv.wgrad1x1 (mivod's kernel from 128 channels, else the
    backward-weights solver); the input gradient is computed
    at the OUTPUT resolution as a forward 1x1 conv with the transposed filter and
    parked in x's producer slot with ``stride = s`` — the producer's BN backward
    kernel adds it on the stride grid.  No full-resolution zero-filled gradient
    (MIOpen strided backward-data: fill + scatter) is ever materialised."""

    @staticmethod
    def forward(ctx, x, w, s, slot, shift=None):
        ctx.save_for_backward(x, w)
        ctx.s, ctx.slot = s, slot
        from .conv import dgrad_filter
        ctx.wt = dgrad_filter(w)
        # the strided 1x1 conv on the 256 x 256 GEMM (rows gathered at the stride) with the
        # following BN's statistics in its epilogue, when it covers the shape
        r = K.native().conv1x1_strided_stats(x, w, s, shift) if _GEMM256 else None
        if r is None:
            z, part = F.conv2d(x, w, None, s), torch.empty(0, device=x.device)
        else:
            z, part = r[0], (r[1] if shift is not None else torch.empty(0, device=x.device))
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return z, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return None, None, None, None, None
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dw = None
        if ctx.needs_input_grad[0]:
            from .conv import dgrad1x1
            assert ctx.slot.grad is None, "a tapped output has one shortcut consumer"
            ctx.slot.grad = dgrad1x1(dy, w, ctx.wt).contiguous(memory_format=torch.channels_last)
            ctx.slot.stride = ctx.s
            ctx.slot.full_shape = x.shape
        if ctx.needs_input_grad[1]:
            from .conv import wgrad1x1
            dw = wgrad1x1(dy, x, w, ctx.s)
        return None, dw, None, None, None


def downsample_tap(x: torch.Tensor, conv: nn.Conv2d, shift=None):
    """``conv(tap(x))`` for a 1x1 strided shortcut conv, fused as _DownsampleTapConv
    when x's producer reads strided second gradients (fused BN, mode 2).  With ``shift``
    (the following BN's running mean) returns ``(z, partials)``: the conv on the 256 x 256
    strided GEMM with that BN's statistics in its epilogue, partials None when it does not
    cover the shape."""
    slot = getattr(x, "_mv_slot", None)
    s = conv.stride[0]
    if (slot is None or not (torch.is_grad_enabled() and x.requires_grad)
            or os.environ.get("MIVOD_BN_TAP", "1") == "0"
            or os.environ.get("MIVOD_DOWNSAMPLE_TAP", "1") == "0"
            or tuple(conv.kernel_size) != (1, 1) or conv.stride[1] != s or s == 1
            or tuple(conv.padding) != (0, 0) or conv.bias is not None or conv.groups != 1
            or x.dtype != torch.bfloat16 or conv.weight.dtype != torch.bfloat16
            or not x.is_contiguous(memory_format=torch.channels_last)):
        z = conv(tap(x))
        return z if shift is None else (z, None)
    z, part = _DownsampleTapConv.apply(x, conv.weight, s, slot, shift)
    if shift is None:
        return z
    return z, (part if part.numel() else None)


def tap(x: torch.Tensor) -> torch.Tensor:
    """Second use of a fused op's output whose gradient the producer adds itself."""
    slot = getattr(x, "_mv_slot", None)
    if slot is None or not (torch.is_grad_enabled() and x.requires_grad) or \
            os.environ.get("MIVOD_BN_TAP", "1") == "0":
        return x
    return _Tap.apply(x, slot)


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu, residual,
                slot, stats=None, colsum=False):
        nat = K.native()
        mode = 2 if (relu and residual is not None) else (1 if relu else 0)
        if stats is not None and mode == 1 and colsum and slot is not None:
            vec = nat.bn_finalize(stats, weight, bias, running_mean, running_var, momentum, eps,
                                  x.numel() // x.shape[1])
            y, slot.colsum = nat.bn_apply_colsum(x, vec[2], vec[3])
            keep = None
        elif stats is not None:
            # statistics came from the producing 1x1 conv's GEMM epilogue (ops.conv)
            if mode == 2 and _BN_MASK:
                y, vec, keep = nat.bn_fwd_train_stats(x, stats, weight, bias, running_mean,
                                                      running_var, momentum, eps, True, residual,
                                                      True)
                mode = 3
            else:
                y, vec = nat.bn_fwd_train_stats(x, stats, weight, bias, running_mean,
                                                running_var, momentum, eps, relu, residual, False)
                keep = y if mode == 2 else None
        elif mode == 2 and _BN_MASK:
            # add+ReLU: backward reads a 1-bit-per-channel mask of y > 0 (mode 3), not y
            y, vec, keep = nat.bn_fwd_train_mask(x, weight, bias, running_mean, running_var,
                                                 momentum, eps, residual)
            mode = 3
        else:
            y, vec = nat.bn_fwd_train(x, weight, bias, running_mean, running_var, momentum, eps,
                                      relu, residual)
            keep = y if mode == 2 else None
        ctx.mode = mode
        ctx.has_res = residual is not None
        ctx.slot = slot
        ctx.save_for_backward(x, keep, vec, weight)
        if slot is not None and mode in (1, 3):
            slot.bn = (x, keep, vec)
            slot.mode = mode
            ctx.set_materialize_grads(False)    # dy is None when a consumer took the reduce
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, vec, weight = ctx.saved_tensors
        need_affine = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        pending = None
        if ctx.slot is not None:
            ctx.slot.bn = None
            pending, ctx.slot.pending = ctx.slot.pending, None
        if pending is not None:
            # the consumer conv's dgrad GEMM already produced dz (masked, shortcut
            # gradient included) and the reduce partials (ops.conv._Conv1x1BN)
            dz, part = pending
            assert ctx.slot.grad is None, "a tapped output has one shortcut consumer"
            if dy is None:
                dx, dg, db = K.native().bn_bwd_from_partials(dz, x, vec, weight, need_affine, part)
            elif ctx.mode == 3:   # a further consumer: d = mask ? dy + dz : 0 (dz is masked)
                dx, dg, db, dz = K.native().bn_bwd(3, _cl(dy), x, y, vec, weight, need_affine,
                                                   dz, 1)
            else:                 # mode 1: relu'(x) (dy + dz) = relu'(x) dy + dz
                dx, dg, db, _ = K.native().bn_bwd(1, _cl(dy) + dz, x, None, vec, weight,
                                                  need_affine, None, 1)
            return (dx if ctx.needs_input_grad[0] else None,
                    dg if ctx.needs_input_grad[1] else None,
                    db if ctx.needs_input_grad[2] else None,
                    None, None, None, None, None, dz if ctx.needs_input_grad[8] else None,
                    None, None, None)
        dy = _cl(dy) if dy is not None else torch.zeros_like(x)
        dy2, s2 = None, 1
        if ctx.slot is not None:
            dy2, s2 = ctx.slot.take_strided() if ctx.mode >= 2 else (ctx.slot.take(), 1)
        if dy2 is not None and ctx.mode < 2:
            dy, dy2 = dy + dy2, None
        dx, dg, db, dz = K.native().bn_bwd(ctx.mode, dy, x, y, vec, weight, need_affine, dy2, s2)
        dres = None
        if ctx.has_res and ctx.needs_input_grad[8]:
            dres = dz if ctx.mode >= 2 else dy
        return (dx if ctx.needs_input_grad[0] else None,
                dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, dres, None, None, None)


def batch_norm_act(x, weight, bias, running_mean, running_var, training, momentum, eps,
                   relu=False, residual=None, stats=None, colsum=False):
    """Functional form: ``act(batch_norm(x) + residual)``.  ``stats``: [P, 2, C]
    statistics partials of x around ``running_mean`` from the producing conv's
    GEMM epilogue (training only; skips the statistics pass)."""
    if _fusable(x, weight) and (residual is None or (residual.dtype == torch.bfloat16 and
                                                     residual.shape == x.shape)):
        if residual is not None:
            residual = _cl(residual)
        if training:
            # mode 2/3: shortcut-gradient taps + fused consumer reduce; mode 1: fused reduce
            slot = GradSlot() if relu else None
            y = _BNActTrain.apply(x, weight, bias, running_mean, running_var, float(momentum),
                                  float(eps), bool(relu), residual, slot, stats, bool(colsum))
            if slot is not None:
                y._mv_slot = slot
            return y
        if not (torch.is_grad_enabled() and (x.requires_grad or (weight is not None and
                                                                 weight.requires_grad))):
            inv = torch.rsqrt(running_var.float() + eps)
            scale = inv * (weight if weight is not None else 1.0)
            shift = (bias if bias is not None else 0.0) - running_mean.float() * scale
            return K.native().bn_apply(x, scale.contiguous(), shift.contiguous(), bool(relu),
                                       residual)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d with a fused ``forward(x, residual=None, relu=False)``."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._mv_steps = 0   # host-side num_batches_tracked (saves a GPU add per call)

    def _train_momentum(self) -> float:
        """Momentum of this training forward (counts the step, as forward does)."""
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats:
            self._mv_steps += 1
            if self.momentum is None:
                momentum = 1.0 / float(self._mv_steps + int(self.num_batches_tracked.item()))
        return momentum

    def forward(self, x, residual=None, relu=False, stats=None, colsum=False):
        self._check_input_dim(x)
        momentum = self._train_momentum()
        bn_training = self.training or (self.running_mean is None and self.running_var is None)
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        if stats is not None and not (self.training and self.track_running_stats):
            stats = None
        return batch_norm_act(x, self.weight, self.bias, rm, rv, bn_training, momentum, self.eps,
                              relu, residual, stats, colsum)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        if self._mv_steps and self.num_batches_tracked is not None:
            with torch.no_grad():
                self.num_batches_tracked.add_(self._mv_steps)
            self._mv_steps = 0
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, *args, **kwargs):
        self._mv_steps = 0
        super()._load_from_state_dict(*args, **kwargs)


# ------------------------------------------------------------------ pooling
class _BNReluMaxPool(torch.autograd.Function):
    """maxpool(relu(bn(x))) for the ResNet stem: statistics pass, then ONE
    kernel applies BN + ReLU and pools (the full-resolution BN output is never
    written); backward: gather-form maxpool backward, then BN+ReLU backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, k, s, p, slot,
                stats=None):
        nat = K.native()
        if stats is not None:       # from the stem conv's epilogue (ops.conv.stem_conv_stats)
            vec = nat.bn_finalize(stats, weight, bias, running_mean, running_var, momentum, eps,
                                  x.numel() // x.shape[1])
        else:
            vec = nat.bn_stats(x, weight, bias, running_mean, running_var, momentum, eps)
        y, idx = nat.maxpool_fwd(x, vec[2], vec[3], True, k, s, p)
        ctx.save_for_backward(x, vec, weight, idx, y)
        ctx.win, ctx.slot = (k, s, p), slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, vec, weight, idx, y = ctx.saved_tensors
        nat = K.native()
        k, s, p = ctx.win
        need_affine = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        if (_POOL_BN_BWD and (k, s, p) == (3, 2, 1) and x.shape[2] % 2 == 0
                and x.shape[3] % 2 == 0 and y.shape[2] * 2 == x.shape[2]
                and y.shape[3] * 2 == x.shape[3] and x.shape[1] <= 256):
            # the BN+ReLU backward fused into the pool backward: reduce over the pooled
            # tensors, then one full-resolution pass (no intermediate pool gradient)
            dx, dg, db = nat.maxpool_bn_bwd(_cl(dy), ctx.slot.take(), idx, y, x, vec, weight)
        else:
            dmid = nat.maxpool_bwd(_cl(dy), ctx.slot.take(), idx, x.shape[2], x.shape[3], k, s, p)
            dx, dg, db, _ = nat.bn_bwd(1, dmid, x, None, vec, weight, need_affine, None, 1)
        return (dx if ctx.needs_input_grad[0] else None,
                dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, None, None, None)


def _pool_args(pool: nn.MaxPool2d):
    def one(v):
        if isinstance(v, (tuple, list)):
            if len(set(v)) != 1:
                return None
            v = v[0]
        return int(v)
    k, s, p = one(pool.kernel_size), one(pool.stride or pool.kernel_size), one(pool.padding)
    ok = (None not in (k, s, p) and one(pool.dilation) == 1 and not pool.ceil_mode
          and not pool.return_indices)
    return (k, s, p) if ok else None


def bn_relu_maxpool(x: torch.Tensor, bn: "BatchNorm2d", pool: nn.MaxPool2d,
                    stats=None) -> torch.Tensor:
    """``pool(relu(bn(x)))``; fused on GPU in training mode.  ``stats``: [P, 2, C]
    statistics partials of x around the BN's running mean from x's producer."""
    win = _pool_args(pool)
    if (bn.training and bn.track_running_stats and win is not None and
            _fusable(x, bn.weight) and bn.weight is not None):
        bn._mv_steps += 1
        momentum = bn.momentum
        if momentum is None:
            momentum = 1.0 / float(bn._mv_steps + int(bn.num_batches_tracked.item()))
        slot = GradSlot()
        y = _BNReluMaxPool.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                 float(momentum), float(bn.eps), *win, slot, stats)
        y._mv_slot = slot
        return y
    return pool(bn(x, relu=True))


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return K.native().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return K.native().gap_bwd(dy.to(torch.bfloat16).contiguous(), *ctx.hw)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``flatten(adaptive_avg_pool2d(x, 1), 1)`` -> [N, C]."""
    if _fusable(x, None):
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


class _PadChannels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cout):
        ctx.c = x.shape[1]
        return K.native().pad_channels(x, cout)

    @staticmethod
    def backward(ctx, dy):
        return dy[:, :ctx.c].contiguous(memory_format=torch.channels_last), None


def pad_channels(x: torch.Tensor, cout: int) -> torch.Tensor:
    """Zero-pad NHWC channels ``C -> cout`` (bf16 channels_last GPU tensors via the
    ``mv_pool.hip`` kernel; anything else via ``F.pad``)."""
    if x.shape[1] == cout:
        return x
    if (os.environ.get("MIVOD_FUSED_BN", "1") != "0" and x.is_cuda and x.dtype == torch.bfloat16
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)):
        return _PadChannels.apply(x, cout)
    return F.pad(x, (0, 0, 0, 0, 0, cout - x.shape[1])).contiguous(
        memory_format=torch.channels_last if x.is_contiguous(memory_format=torch.channels_last)
        else torch.contiguous_format)


class _Conv1x1BNFold(torch.autograd.Function):
    """``relu(bn(conv1x1(x)) + residual)`` (training, stride 1) with the BN backward folded
    into the conv's backward GEMMs — the BN's input gradient dL/dz is never materialised.

    With z = x W^T and the BN backward dL/dz = ca*dz + cb*z + cc (per output channel;
    ca, cb, cc from the finalize of the reduce partials that the consuming conv's
    data-gradient epilogue produced, ``slot.pending``; dz = the masked output gradient):
        dx = dz (diag(ca) W) + x (W^T diag(cb) W) + cc W
        dW = diag(ca) (dz^T x) + diag(cb) W (x^T x) + cc (x) colsum(x)
    so the backward is ONE dual-source GEMM for dx ([dz | x] . [diag(ca) W ; W^T diag(cb) W]
    + cc W, mv_gemm's EPI 4, which also runs the ReLU backward reduce of BN2 — the producer
    of x — in its epilogue; two hipBLASLt GEMMs on shapes it does not cover), mivod's
    wgrad1x1 kernel for dz^T x and the Gram matrix x^T x (fp32 out), and a few p x p /
    4p x p products — instead of the BN dx pass (read dz, z; write dL/dz) + dgrad + wgrad
    of dL/dz.  Forward (``_RECOMPUTE``): z is never written — a statistics-only GEMM pass,
    the finalize, then the GEMM again with the BN+add+ReLU apply in its epilogue.  The
    consumer's epilogue reduce only sums dz (``slot.fold``: z is not read there either);
    sum dz (z - mean) = sum_k W[c, k] (dz^T x)[c, k] - mean * sum dz.  When no
    consumer supplied the reduce (the stage's last blocks feeding a plain conv or the
    pooling head) it runs the unfused BN backward and conv backward.
    ``MIVOD_BN_FOLD=0`` disables it (A/B)."""

    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, momentum, eps, residual,
                slot, gemm, res_w=None, res_b=None, res_cfg=None, res_conv_w=None):
        nat = K.native()
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        vec_r = None
        sfold = res_conv_w is not None
        ctx.sfold = sfold
        if res_cfg is not None:
            # projection shortcut: residual is the shortcut BN's INPUT (or, sfold, the
            # shortcut CONV's input); its statistics come from the shortcut conv's GEMM
            # epilogue (or a statistics pass) and its apply runs inside this GEMM's
            # epilogue (conv_bn(..., res_bn=))
            assert gemm and _RECOMPUTE and nat.gemm_apply_supported(cout, cin)
            rm_r, rv_r, mom_r, eps_r, part_r = res_cfg[:5]
            if sfold:
                s_r, ctx.x0slot = res_cfg[5], res_cfg[6]
                ctx.s_r = s_r
                c0 = residual.shape[1]
                dual = None
                if (s_r == 1 and _SHORTCUT_DUAL and c0 == cin
                        and nat.gemm_apply_dual_supported(cout, cin)):
                    # z_sc is never written: statistics-only pass here, recomputed in the
                    # apply GEMM below (EPI 7)
                    m0 = n * h * wd
                    dual = (residual.permute(0, 2, 3, 1).reshape(m0, c0),
                            res_conv_w.permute(0, 2, 3, 1).reshape(cout, c0))
                    part_r = torch.empty(nat.gemm_partials(m0, cout, c0), 2, cout,
                                         dtype=torch.float32, device=x.device)
                    nat.gemm_nt(dual[0], dual[1], None, rm_r, part_r)
                    zr_in = None
                elif s_r == 1 and c0 in (64, 128, 256):
                    m0 = n * h * wd
                    zrf = torch.empty(m0, cout, dtype=x.dtype, device=x.device)
                    part_r = torch.empty(nat.gemm_partials(m0, cout, c0), 2, cout,
                                         dtype=torch.float32, device=x.device)
                    nat.gemm_nt(residual.permute(0, 2, 3, 1).reshape(m0, c0),
                                res_conv_w.permute(0, 2, 3, 1).reshape(cout, c0), zrf, rm_r,
                                part_r)
                    zr_in = zrf.view(n, h, wd, cout).permute(0, 3, 1, 2)
                else:
                    # strided shortcut conv + its BN statistics on the 256 x 256 GEMM
                    # (rows gathered at the stride: no strided copy of the block input)
                    r = (nat.conv1x1_strided_stats(residual, res_conv_w, s_r, rm_r)
                         if _GEMM256 else None)
                    if r is not None:
                        zr_in, part_r = r[0], r[1]
                    else:
                        zr_in = _cl(F.conv2d(residual, res_conv_w, None, s_r))
                        part_r = None
            else:
                zr_in, dual = residual, None
            if part_r is not None:
                vec_r = nat.bn_finalize(part_r, res_w, res_b, rm_r, rv_r, mom_r, eps_r,
                                        n * h * wd)
            else:
                vec_r = nat.bn_stats(zr_in, res_w, res_b, rm_r, rv_r, mom_r, eps_r)
            residual_in = zr_in
        else:
            residual_in, dual = residual, None
        if (gemm and _RECOMPUTE and nat.gemm_apply_supported(cout, cin)
                and (res_cfg is not None or cin <= _RECOMPUTE_MAXK)):
            # z is never materialised: a statistics-only GEMM pass, the finalize, then the
            # GEMM again with relu(bn(z) + residual) and the bitmask in its epilogue (the
            # same tile order, so z and y are bit-identical to the two-pass path).  The
            # expansion conv's z is the widest activation of the block: writing it and
            # re-reading it in the apply pass costs more than a second K <= 256 GEMM.
            m = n * h * wd
            x2 = x.permute(0, 2, 3, 1).reshape(m, cin)
            w2 = w.permute(0, 2, 3, 1).reshape(cout, cin)
            xcs = getattr(getattr(x, "_mv_slot", None), "colsum", None)
            if (_GRAM_STATS and xcs is not None and cin % 64 == 0 and cin <= 1024
                    and cout % 16 == 0):
                part = _gram_stats(nat, x, w2, xcs, running_mean, m)
            else:
                part = torch.empty(nat.gemm_partials(m, cout, cin), 2, cout,
                                   dtype=torch.float32, device=x.device)
                nat.gemm_nt(x2, w2, None, running_mean, part)
            vec = nat.bn_finalize(part, weight, bias, running_mean, running_var, momentum, eps, m)
            if dual is not None:
                yf, keep = nat.gemm_nt_apply_dual(x2, w2, dual[0], dual[1], vec[2], vec[3],
                                                  vec_r[2], vec_r[3])
            else:
                yf, keep = nat.gemm_nt_apply(x2, w2,
                                             residual_in.permute(0, 2, 3, 1).reshape(m, cout),
                                             vec[2], vec[3], None if vec_r is None else vec_r[2],
                                             None if vec_r is None else vec_r[3])
            y = yf.view(n, h, wd, cout).permute(0, 3, 1, 2)
            z = None
        elif gemm:
            m = n * h * wd
            zf = torch.empty(m, cout, dtype=x.dtype, device=x.device)
            part = torch.empty(nat.gemm_partials(m, cout, cin), 2, cout, dtype=torch.float32,
                               device=x.device)
            nat.gemm_nt(x.permute(0, 2, 3, 1).reshape(m, cin),
                        w.permute(0, 2, 3, 1).reshape(cout, cin), zf, running_mean, part)
            z = zf.view(n, h, wd, cout).permute(0, 3, 1, 2)
            y, vec, keep = nat.bn_fwd_train_stats(z, part, weight, bias, running_mean, running_var,
                                                  momentum, eps, True, residual, True)
        else:
            z = F.conv2d(x, w)
            y, vec, keep = nat.bn_fwd_train_mask(z, weight, bias, running_mean, running_var,
                                                 momentum, eps, residual)
        ctx.save_for_backward(x, w, z, keep, vec, weight, vec_r, res_w,
                              residual if vec_r is not None else None, res_conv_w)
        ctx.slot = slot
        from .conv import dgrad_filter
        ctx.wt = dgrad_filter(w)
        ctx.xslot = getattr(x, "_mv_slot", None)     # x = relu(bn2(z2)): BN2's GradSlot
        ctx.colsum = getattr(ctx.xslot, "colsum", None)
        slot.bn = (z, keep, vec)
        slot.mode = 3
        slot.fold = True
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .conv import dgrad1x1, wgrad1x1
        x, w, z, keep, vec, weight, vec_r, res_w, zr, res_conv_w = ctx.saved_tensors
        slot = ctx.slot
        slot.bn = None
        pending, slot.pending = slot.pending, None
        nat = K.native()
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        fold_part = None
        if pending is not None and dy is None:
            dz, part = pending
            assert slot.grad is None, "a tapped output has one shortcut consumer"
            n, cin, h, wd = x.shape
            cout, m = w.shape[0], n * h * wd
            x2 = x.permute(0, 2, 3, 1).reshape(m, cin)
            if need_w and _DUAL_WGRAD:
                # dz^T x and the Gram x^T x in one pass over x: [dz | x]^T . x
                gg = nat.wgrad1x1(x, dz, 1, True, x).view(cout + cin, cin)
                g, gram = gg[:cout], gg[cout:]
            else:
                g = nat.wgrad1x1(x, dz, 1, True).view(cout, cin)          # dz^T x
                gram = nat.wgrad1x1(x, x, 1, True).view(cin, cin) if need_w else None
            # the consumer's epilogue summed dz only (part); colsum(x) from BN2's apply pass
            dg, db, dwb, bcat, badd = _fold_math(
                nat, w.reshape(cout, cin), g, gram, vec, weight, m, part, None, ctx.colsum,
                lambda: nat.bn_stats(x, None, None, None, None, 0.0, 0.0)[0] * float(m), need_w)
            fold_part = part
            if need_w:
                dw = dwb.view(cout, cin, 1, 1)
            xs = ctx.xslot
            if (need_x and _FOLD_DX and xs is not None and xs.bn is not None and xs.mode == 1
                    and xs.pending is None and nat.gemm_fold_dx_partials(m, cout, cin) > 0):
                # one dual-source GEMM [dz | x] . [diag(ca) W ; W^T diag(cb) W] + cc W with
                # BN2's ReLU backward reduce in its epilogue: BN2 (the producer of x) gets
                # (d, partials) through its slot and autograd gets None for x
                zb, _, vec2 = xs.bn
                d = torch.empty_like(zb)
                part2 = nat.gemm_fold_dx(dz.permute(0, 2, 3, 1).reshape(m, cout), x2, bcat, badd,
                                         d.permute(0, 2, 3, 1).reshape(m, cin),
                                         zb.permute(0, 2, 3, 1).reshape(m, cin), vec2)
                xs.pending = (d, part2)
            elif need_x:
                dx2 = torch.addmm(badd.to(x.dtype), dz.permute(0, 2, 3, 1).reshape(m, cout),
                                  bcat[:, :cout].t())
                dx2.addmm_(x2, bcat[:, cout:].t())
                dx = dx2.view(n, h, wd, cin).permute(0, 3, 1, 2)
        else:
            if z is None:               # recompute forward: rebuild z (same GEMM, same bits)
                n, cin, h, wd = x.shape
                cout, m = w.shape[0], n * h * wd
                zf = torch.empty(m, cout, dtype=x.dtype, device=x.device)
                nat.gemm_nt(x.permute(0, 2, 3, 1).reshape(m, cin),
                            w.permute(0, 2, 3, 1).reshape(cout, cin), zf, None, None)
                z = zf.view(n, h, wd, cout).permute(0, 3, 1, 2)
            if pending is not None:     # a further consumer: d = mask ? dy + dz : 0
                dlz, dg, db, dz = nat.bn_bwd(3, _cl(dy), z, keep, vec, weight, True, pending[0], 1)
            else:
                dy = _cl(dy) if dy is not None else torch.zeros_like(z)
                dy2, s2 = slot.take_strided()
                dlz, dg, db, dz = nat.bn_bwd(3, dy, z, keep, vec, weight, True, dy2, s2)
            if need_x:
                dx = dgrad1x1(dlz, w, ctx.wt)
            if need_w:
                dw = wgrad1x1(dlz, x, w)
        dres = dz if ctx.needs_input_grad[8] else None
        dgr = dbr = dwr = None
        if ctx.sfold:
            # the shortcut conv + BN folded like conv3 + BN3 (zr = the conv's input x0):
            # dz_sc = ca_r dz + cb_r (x0s W_r^T) + cc_r, so dx0 = [dz | x0s] . [diag(ca_r) W_r ;
            # W_r^T diag(cb_r) W_r] + cc_r W_r and dW_r = diag(ca_r) dz^T x0s + diag(cb_r) W_r
            # x0s^T x0s + cc_r colsum(x0s); the BN input z_sc is never read.  dx0 is parked in
            # x0's producer slot (on the stride grid when s > 1), autograd gets None.
            s_r = ctx.s_r
            x0 = zr
            nb, c0 = x0.shape[0], x0.shape[1]
            cout_r = res_conv_w.shape[0]
            # x0s = x0[:, :, ::s, ::s] is never copied on the covered shapes: the kernels
            # below read x0 at the stride grid (the copy is made lazily for the fallbacks)
            x0s_c = [x0 if s_r == 1 else None]

            def x0s():
                if x0s_c[0] is None:
                    x0s_c[0] = _cl(x0[:, :, ::s_r, ::s_r])
                return x0s_c[0]
            ho, wo = (x0.shape[2] - 1) // s_r + 1, (x0.shape[3] - 1) // s_r + 1
            mr = nb * ho * wo
            dzc = _cl(dz)
            need_wr = ctx.needs_input_grad[14]
            if need_wr and _DUAL_WGRAD:      # [dz | x0s]^T . x0s (x0 read at the stride twice)
                gg = nat.wgrad1x1(x0, dzc, s_r, True, x0).view(cout_r + c0, c0)
                gr, gram = gg[:cout_r], gg[cout_r:]
            else:
                gr = nat.wgrad1x1(x0, dzc, s_r, True).view(cout_r, c0)          # dz^T x0s
                gram = nat.wgrad1x1(x0s(), x0s(), 1, True).view(c0, c0) if need_wr else None
            # same dz as the main branch: its consumer's partials give sum dz
            part_r = fold_part
            sdz_r = None if part_r is not None else torch.sum(dzc, (0, 2, 3), dtype=torch.float32)
            dgr, dbr, dwrb, bcat, badd = _fold_math(
                nat, res_conv_w.reshape(cout_r, c0), gr, gram, vec_r, res_w, mr, part_r, sdz_r,
                None, lambda: nat.bn_stats_strided(x0, s_r)[0] * float(mr), need_wr)
            if need_wr:
                dwr = dwrb.view(cout_r, c0, 1, 1)
            dz2d = dzc.permute(0, 2, 3, 1).reshape(mr, cout_r)
            d0 = torch.empty(mr, c0, dtype=x0.dtype, device=x0.device)
            if s_r > 1 and nat.gemm_dual_bias_strided(dz2d, x0, s_r, bcat, badd, d0):
                pass
            elif nat.gemm_dual_supported(cout_r, c0):
                nat.gemm_dual_bias(dz2d, x0s().permute(0, 2, 3, 1).reshape(mr, c0), bcat, badd, d0)
            else:
                x02d = x0s().permute(0, 2, 3, 1).reshape(mr, c0)
                d0 = torch.addmm(badd.to(x0.dtype), dz2d, bcat[:, :cout_r].t())
                d0.addmm_(x02d, bcat[:, cout_r:].t())
            d0 = d0.view(nb, ho, wo, c0).permute(0, 3, 1, 2)
            s0 = ctx.x0slot
            assert s0.grad is None, "a tapped output has one shortcut consumer"
            s0.grad, s0.stride = d0, s_r
            if s_r > 1:
                s0.full_shape = x0.shape
            dres = None
        elif vec_r is not None:
            # the shortcut BN's backward (no activation) on the residual-branch gradient
            dres, dgr, dbr, _ = nat.bn_bwd(0, _cl(dz), _cl(zr), None, vec_r, res_w, True, None, 1)
        return (dx, dw, dg if ctx.needs_input_grad[2] else None,
                db if ctx.needs_input_grad[3] else None, None, None, None, None,
                dres if ctx.needs_input_grad[8] else None, None, None,
                dgr if ctx.needs_input_grad[11] else None,
                dbr if ctx.needs_input_grad[12] else None, None, dwr)


class _BNReluConv64(torch.autograd.Function):
    """``conv3x3(relu(bn1(z1)))`` for the 64 -> 64 stride-1 conv2 of a ResNet-50 layer1
    bottleneck with BN1 + ReLU applied while the row-patch kernels stage their input patch
    (csrc/kernels/mv_conv64.hip): the BN1 output is never written (its apply pass was ~0.28
    ms per block at bs2048) — forward (+ BN2 statistics) and the weight gradient read z1
    and recompute relu(bn1(z1)) on the fly; the data gradient carries BN1's backward reduce
    as before (mask from z1 through BN1's affine).  BN1's statistics come from conv1's GEMM
    epilogue (``part1``); its running statistics update in the finalize.
    ``MIVOD_BN_APPLY_FUSE=0`` keeps the materialised path (A/B)."""

    @staticmethod
    def forward(ctx, z1, part1, g1, b1, rm1, rv1, mom1, eps1, w2, shift2):
        nat = K.native()
        n, _, h, wd = z1.shape
        m = n * h * wd
        vec1 = nat.bn_finalize(part1, g1, b1, rm1, rv1, mom1, eps1, m)
        k = w2.shape[0]
        part2 = torch.empty(nat.conv3x3_partials(m, k), 2, k, dtype=torch.float32,
                            device=z1.device)
        z2 = nat.conv3x3(z1, w2.contiguous(memory_format=torch.channels_last), 1, shift2, part2,
                         vec1[2], vec1[3])
        ctx.save_for_backward(z1, vec1, g1, w2)
        from .conv import dgrad_filter
        ctx.wt = dgrad_filter(w2)
        ctx.mark_non_differentiable(part2)
        ctx.set_materialize_grads(False)
        return z2, part2

    @staticmethod
    def backward(ctx, dz2, _dpart):
        if dz2 is None:
            return (None,) * 10
        from .conv import _wt_or_make
        z1, vec1, g1, w2 = ctx.saved_tensors
        nat = K.native()
        dz2 = _cl(dz2)
        # conv2's data gradient with BN1's ReLU mask and backward reduce in its epilogue
        d1, p1 = nat.conv3x3_bn_bwd(dz2, _wt_or_make(w2, ctx.wt), z1, vec1)
        dw2 = (nat.wgrad3x3(z1, dz2, 1, vec1[2], vec1[3]) if ctx.needs_input_grad[8] else None)
        need_aff = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dz1, dg1, db1 = nat.bn_bwd_from_partials(d1, z1, vec1, g1, need_aff, p1)
        return (dz1 if ctx.needs_input_grad[0] else None, None,
                dg1 if ctx.needs_input_grad[2] else None,
                db1 if ctx.needs_input_grad[3] else None, None, None, None, None, dw2, None)


def bn_relu_conv3x3(conv1: nn.Conv2d, bn1: "BatchNorm2d", conv2: nn.Conv2d, bn2: "BatchNorm2d",
                    x: torch.Tensor):
    """``(z2, BN2 statistics partials)`` of ``conv2(relu(bn1(conv1(x))))`` through
    _BNReluConv64 when it applies (training, 64 -> 64 stride-1 3x3 conv2 on the row-patch
    kernels, conv1 a statistics-fusable 1x1), else None."""
    from .conv import bwd_fusable, conv1x1_bn, stats_fusable
    if (os.environ.get("MIVOD_BN_APPLY_FUSE", "1") == "0" or not torch.is_grad_enabled()
            or not (bn1.training and bn1.track_running_stats and bn2.training
                    and bn2.track_running_stats)
            or bn1.running_mean is None or bn2.running_mean is None or bn1.weight is None
            or bn1.bias is None or not _fusable(x, bn1.weight)
            or conv1.out_channels != 64 or conv2.in_channels != 64 or conv2.out_channels != 64
            or tuple(conv2.kernel_size) != (3, 3) or tuple(conv2.stride) != (1, 1)
            or tuple(conv2.padding) != (1, 1) or tuple(conv2.dilation) != (1, 1)
            or conv2.groups != 1 or conv2.bias is not None
            or conv2.weight.dtype != torch.bfloat16 or not stats_fusable(conv1, x)):
        return None
    n, _, h, w = x.shape
    st = conv1.stride[0]
    h, w = (h - 1) // st + 1, (w - 1) // st + 1
    # the row-patch kernels: forward W <= 62 (8 rows x W <= 448 pixels), weight gradient
    # W % 4 == 0 and W <= 56
    if not (w <= 56 and w % 4 == 0 and h >= 1):
        return None
    z1, part1 = conv1x1_bn(conv1, x, bn1.running_mean, True, bwd_fusable(conv1, x))
    return _BNReluConv64.apply(z1, part1, bn1.weight, bn1.bias, bn1.running_mean,
                               bn1.running_var, float(bn1._train_momentum()), float(bn1.eps),
                               conv2.weight, bn2.running_mean)


def _fold_eligible(conv: nn.Conv2d, bn: "BatchNorm2d", x: torch.Tensor, relu, residual) -> bool:
    from .conv import _eligible
    return (os.environ.get("MIVOD_BN_FOLD", "1") != "0" and relu and residual is not None
            and _BN_MASK and bn.training and bn.track_running_stats
            and bn.running_mean is not None and bn.weight is not None and bn.bias is not None
            and _fusable(x, bn.weight) and residual.dtype == torch.bfloat16
            and torch.is_grad_enabled() and x.requires_grad and _eligible(conv, x)
            and tuple(conv.kernel_size) == (1, 1) and conv.in_channels % 64 == 0
            and conv.out_channels % 64 == 0)


def shortcut_fusable(conv: nn.Conv2d, bn: "BatchNorm2d", x: torch.Tensor,
                     res_bn: nn.Module) -> bool:
    """A projection shortcut's BN (``res_bn``) can be applied inside the epilogue of
    conv3's recomputing GEMM (``conv_bn(conv, bn, x, True, z_shortcut, res_bn=...)``)."""
    from .conv import stats_fusable
    return (_SHORTCUT and _RECOMPUTE and isinstance(res_bn, BatchNorm2d) and res_bn.training
            and res_bn.track_running_stats and res_bn.running_mean is not None
            and res_bn.weight is not None and res_bn.bias is not None
            and res_bn.weight.dtype == torch.float32
            and _fold_eligible(conv, bn, x, True, x) and stats_fusable(conv, x)
            and K.native().gemm_apply_supported(conv.out_channels, conv.in_channels))


def shortcut_foldable(sc_conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """The projection shortcut conv ``sc_conv`` on the block input ``x`` can fold into the
    block's fused backward (plain 1x1, x a fused output with a gradient slot)."""
    return (_SHORTCUT_FOLD and getattr(x, "_mv_slot", None) is not None
            and isinstance(sc_conv, nn.Conv2d) and tuple(sc_conv.kernel_size) == (1, 1)
            and sc_conv.stride[0] == sc_conv.stride[1] and tuple(sc_conv.padding) == (0, 0)
            and sc_conv.bias is None and sc_conv.groups == 1 and tuple(sc_conv.dilation) == (1, 1)
            and sc_conv.weight.dtype == torch.bfloat16 and sc_conv.in_channels % 64 == 0
            and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
            and torch.is_grad_enabled() and x.requires_grad)


def conv_bn(conv: nn.Conv2d, bn: "BatchNorm2d", x: torch.Tensor, relu: bool = False,
            residual=None, res_bn=None, res_part=None, res_conv=None,
            colsum: bool = False) -> torch.Tensor:
    """``bn(conv(x), residual, relu)`` with the BN statistics computed inside the
    1x1 conv's GEMM epilogue when the conv qualifies (ops.conv.stats_fusable) and
    the BN is training with running statistics, and with x's producer BN backward
    reduce run in this conv's data-gradient GEMM when x is a fused BN+add+ReLU output
    (ops.conv.bwd_fusable); the plain composition otherwise."""
    from .conv import (bwd3x3_fusable, bwd_fusable, conv1x1_bn, conv3x3_bn, conv3x3_eligible,
                       stats_fusable)
    train_stats = (bn.training and bn.track_running_stats and bn.running_mean is not None
                   and _fusable(x, bn.weight))
    if res_bn is not None:
        # residual = the projection shortcut conv's output; res_bn = its BN (res_part: that
        # BN's statistics partials from the shortcut GEMM's epilogue, or None)
        # (res_conv: residual is that conv's INPUT, folded into this block's backward)
        if res_conv is not None:
            if shortcut_fusable(conv, bn, x, res_bn) and shortcut_foldable(res_conv, residual):
                slot = GradSlot()
                cfg = (res_bn.running_mean, res_bn.running_var, float(res_bn._train_momentum()),
                       float(res_bn.eps), None, res_conv.stride[0], residual._mv_slot)
                y = _Conv1x1BNFold.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean,
                                         bn.running_var, float(bn._train_momentum()),
                                         float(bn.eps), residual, slot, True, res_bn.weight,
                                         res_bn.bias, cfg, res_conv.weight)
                y._mv_slot = slot
                return y
            residual = res_bn(res_conv(tap(residual)))
            res_bn = None
    if res_bn is not None:
        residual = _cl(residual)
        if (shortcut_fusable(conv, bn, x, res_bn) and residual.shape[0] == x.shape[0]
                and residual.shape[1] == conv.out_channels):
            slot = GradSlot()
            cfg = (res_bn.running_mean, res_bn.running_var, float(res_bn._train_momentum()),
                   float(res_bn.eps), res_part)
            y = _Conv1x1BNFold.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean,
                                     bn.running_var, float(bn._train_momentum()), float(bn.eps),
                                     residual, slot, True, res_bn.weight, res_bn.bias, cfg, None)
            y._mv_slot = slot
            return y
        residual = res_bn(residual, stats=res_part)
    if _fold_eligible(conv, bn, x, relu, residual):
        residual = _cl(residual)
        if residual.shape[0] == x.shape[0] and residual.shape[1] == conv.out_channels:
            slot = GradSlot()
            y = _Conv1x1BNFold.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean,
                                     bn.running_var, float(bn._train_momentum()), float(bn.eps),
                                     residual, slot, stats_fusable(conv, x), None, None, None,
                                     None)
            y._mv_slot = slot
            return y
    if conv3x3_eligible(conv, x):
        y, part = conv3x3_bn(conv, x, bn.running_mean if train_stats else None, train_stats,
                             bwd3x3_fusable(conv, x))
        return bn(y, residual=residual, relu=relu, stats=part if train_stats else None,
                  colsum=colsum and _COLSUM)
    fwd = train_stats and stats_fusable(conv, x)
    slot = bwd_fusable(conv, x)
    if fwd or slot is not None:
        y, part = conv1x1_bn(conv, x, bn.running_mean if fwd else None, fwd, slot)
        return bn(y, residual=residual, relu=relu, stats=part if fwd else None)
    return bn(conv(x), residual=residual, relu=relu)
