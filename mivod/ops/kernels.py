"""Python entry points for the hand-written gfx950 kernels (``mivod._mvk``).

GPU tensors always go to the HIP kernels; if the extension is missing on a GPU
process this module raises instead of silently falling back.  CPU tensors (the
gloo test tier) use the plain-PyTorch reference implementations below, which
are also the fp32 references the numerics tests compare the kernels against.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

try:
    from .. import _mvk  # type: ignore
    _IMPORT_ERROR = None
except Exception as e:  # pragma: no cover - exercised when not built
    _mvk = None
    _IMPORT_ERROR = e

CHUNK = 4096


def available() -> bool:
    return _mvk is not None


def native():
    """Return the native module or raise loudly (GPU path must be native)."""
    if _mvk is None:
        raise RuntimeError(
            "mivod HIP kernels (mivod/_mvk*.so) are not built/loadable: "
            f"{_IMPORT_ERROR!r}. Run `python -m mivod._build`.")
    return _mvk


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ---------------------------------------------------------------------------
# K1/K2 pack / unpack
# ---------------------------------------------------------------------------
def pack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int],
         scale: float = 1.0, nonfinite: Optional[torch.Tensor] = None) -> None:
    """flat[off_i : off_i+n_i] = cast(t_i * scale) for every tensor (raw memory
    order of t_i).  Tensors of one call must share a dtype."""
    if not tensors:
        return
    if _on_gpu(flat):
        native().mt_copy(list(tensors), flat, [int(o) for o in offsets], True, float(scale),
                         nonfinite)
        return
    for t, o in zip(tensors, offsets):
        src = _raw_flat(t)
        dst = flat[o:o + src.numel()]
        v = src.float() * scale if scale != 1.0 else src
        if nonfinite is not None and not bool(torch.isfinite(v.float()).all()):
            nonfinite.fill_(1)
        dst.copy_(v)


def unpack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int],
           scale: float = 1.0) -> None:
    """t_i (raw memory order) = cast(flat[off_i : off_i+n_i] * scale)."""
    if not tensors:
        return
    if _on_gpu(flat):
        native().mt_copy(list(tensors), flat, [int(o) for o in offsets], False, float(scale), None)
        return
    for t, o in zip(tensors, offsets):
        dst = _raw_flat(t)
        src = flat[o:o + dst.numel()]
        dst.copy_(src.float() * scale if scale != 1.0 else src)


def is_dense(t: torch.Tensor) -> bool:
    """True when ``t`` covers exactly numel() contiguous elements in some dim
    order (contiguous, channels_last, any permutation)."""
    if t.is_contiguous():
        return True
    dims = sorted((d for d in range(t.dim()) if t.size(d) != 1), key=lambda d: t.stride(d))
    expect = 1
    for d in dims:
        if t.stride(d) != expect:
            return False
        expect *= t.size(d)
    return True


def _raw_flat(t: torch.Tensor) -> torch.Tensor:
    """1-D view of a dense tensor in its memory order (channels_last aware)."""
    if t.is_contiguous():
        return t.view(-1)
    if not is_dense(t):
        raise ValueError("mivod pack/unpack needs dense tensors")
    # permute to memory order, which is contiguous
    perm = sorted(range(t.dim()), key=lambda d: (-t.stride(d), d))
    return t.permute(*perm).reshape(-1)


def flat_cast(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0,
              nonfinite: Optional[torch.Tensor] = None) -> None:
    """dst = cast(src * scale); src and dst may alias (in-place scale)."""
    if _on_gpu(src):
        native().flat_cast(src, dst, float(scale), nonfinite)
        return
    v = src.float() * scale
    if nonfinite is not None and not bool(torch.isfinite(v).all()):
        nonfinite.fill_(1)
    dst.copy_(v)


def nonfinite_scan(x: torch.Tensor, flag: torch.Tensor) -> None:
    """flag |= any non-finite element of ``x`` (read-only; the overflow guard's
    per-bucket check of the REDUCED gradient)."""
    if _on_gpu(x):
        native().nonfinite_scan(x, flag)
        return
    if not bool(torch.isfinite(x.float()).all()):
        flag.fill_(1)


# ---------------------------------------------------------------------------
# K6 fused optimizers (flat)
# ---------------------------------------------------------------------------
def _skipped(skip) -> bool:
    return skip is not None and int(skip.reshape(-1)[0]) != 0


def sgd_step(g, w, mom, model, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0,
             gscale=1.0, nesterov=False, first=False, dyn=None, skip=None):
    """``dyn`` (GPU only): device fp32 [lr, first, bc1, bc2] read by the kernel in
    place of ``lr`` / ``first`` — the HIP-graph replay path (mivod.torch.graphs).
    ``skip``: device int32 flag; nonzero => no update (fp16-wire overflow guard)."""
    if _on_gpu(g):
        native().sgd_step(g, w, mom, model, float(lr), float(momentum), float(dampening),
                          float(weight_decay), float(gscale), bool(nesterov), bool(first), dyn,
                          skip)
        return
    if _skipped(skip):
        return
    d = g.float() * gscale + weight_decay * w
    if mom is not None:
        if first:
            mom.copy_(d)
        else:
            mom.mul_(momentum).add_(d, alpha=1.0 - dampening)
        d = d + momentum * mom if nesterov else mom
    w.sub_(lr * d)
    if model is not None:
        model.copy_(w)


def adam_step(g, w, m, v, model, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
              gscale=1.0, step=1, adamw=False, keras_eps=False, dyn=None, skip=None):
    if _on_gpu(g):
        native().adam_step(g, w, m, v, model, float(lr), float(beta1), float(beta2), float(eps),
                           float(weight_decay), float(gscale), int(step), bool(adamw),
                           bool(keras_eps), dyn, skip)
        return
    if _skipped(skip):
        return
    gr = g.float() * gscale
    if not adamw and weight_decay:
        gr = gr + weight_decay * w
    m.mul_(beta1).add_(gr, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gr, gr, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    if adamw and weight_decay:
        w.mul_(1 - lr * weight_decay)
    if keras_eps:
        denom = (v.sqrt() + eps) / math.sqrt(bc2)
    else:
        denom = v.sqrt() / math.sqrt(bc2) + eps
    w.addcdiv_(m, denom, value=-lr / bc1)
    if model is not None:
        model.copy_(w)


def adadelta_step(g, w, sq, acc, model, *, lr=1.0, rho=0.9, eps=1e-6, weight_decay=0.0,
                  gscale=1.0, dyn=None, skip=None):
    if _on_gpu(g):
        native().adadelta_step(g, w, sq, acc, model, float(lr), float(rho), float(eps),
                               float(weight_decay), float(gscale), dyn, skip)
        return
    if _skipped(skip):
        return
    gr = g.float() * gscale + weight_decay * w
    sq.mul_(rho).addcmul_(gr, gr, value=1 - rho)
    delta = (acc + eps).sqrt() / (sq + eps).sqrt() * gr
    acc.mul_(rho).addcmul_(delta, delta, value=1 - rho)
    w.sub_(lr * delta)
    if model is not None:
        model.copy_(w)


# ---------------------------------------------------------------------------
# Segment / chunk tables (LARS, Adasum)
# ---------------------------------------------------------------------------
@dataclass
class ChunkTable:
    seg_sizes: list
    begin: torch.Tensor
    len: torch.Tensor
    seg: torch.Tensor
    seg_c0: torch.Tensor
    seg_nc: torch.Tensor
    seg_offsets: list
    total: int
    # derived tables (e.g. Adasum's per-level clipped ranges), owned by this
    # table so they can never outlive it or be served to another table
    derived: dict = field(default_factory=dict, repr=False, compare=False)

    @property
    def nchunks(self) -> int:
        return self.begin.numel()

    @property
    def nseg(self) -> int:
        return len(self.seg_sizes)


def make_chunk_table(seg_sizes: Sequence[int], device, seg_offsets: Optional[Sequence[int]] = None,
                     chunk: int = CHUNK) -> ChunkTable:
    """Chunk table of a flat buffer made of consecutive segments (optionally at
    explicit offsets, e.g. 64-element-aligned arena slots)."""
    if seg_offsets is None:
        seg_offsets, o = [], 0
        for s in seg_sizes:
            seg_offsets.append(o)
            o += s
    begin, ln, sg, c0, nc = [], [], [], [], []
    for i, (s, off) in enumerate(zip(seg_sizes, seg_offsets)):
        c0.append(len(begin))
        n = 0
        for b in range(0, max(int(s), 1), chunk):
            begin.append(int(off) + b)
            ln.append(int(min(chunk, s - b)) if s > 0 else 0)
            sg.append(i)
            n += 1
        nc.append(n)
    total = max((o + s for o, s in zip(seg_offsets, seg_sizes)), default=0)
    dev = torch.device(device)
    return ChunkTable(list(map(int, seg_sizes)),
                      torch.tensor(begin, dtype=torch.int64, device=dev),
                      torch.tensor(ln, dtype=torch.int32, device=dev),
                      torch.tensor(sg, dtype=torch.int32, device=dev),
                      torch.tensor(c0, dtype=torch.int32, device=dev),
                      torch.tensor(nc, dtype=torch.int32, device=dev),
                      list(map(int, seg_offsets)), int(total))


def _check_table(table: ChunkTable, numel: int) -> None:
    """Host-side bound check before a segmented launch: every chunk of the
    table must lie inside the buffers the kernel will index."""
    if table.total > numel:
        raise ValueError(f"mivod: chunk table covers {table.total} elements but the buffer "
                         f"has {numel}")


def lars_step(g, w, mom, model, table: ChunkTable, seg_flags: torch.Tensor, *, lr, momentum=0.9,
              weight_decay=0.0, eta=0.001, gscale=1.0, eps=0.0, first=False,
              workspace: Optional[dict] = None, dyn=None, skip=None):
    """Segmented LARS (You et al. 2017): per segment trust = eta*|w|/(|g|+wd*|w|);
    flagged segments (bit0) get trust 1 and no weight decay."""
    _check_table(table, g.numel())
    if _on_gpu(g):
        ws = workspace if workspace is not None else {}
        partial = ws.get("partial")
        if partial is None or partial.numel() < 2 * table.nchunks:
            partial = ws["partial"] = torch.empty(2 * table.nchunks, dtype=torch.float32,
                                                  device=g.device)
        norms = ws.get("norms")
        if norms is None or norms.numel() < 2 * table.nseg:
            norms = ws["norms"] = torch.empty(2 * table.nseg, dtype=torch.float32, device=g.device)
        native().lars_step(g, w, mom, model, table.begin, table.len, table.seg, table.seg_c0,
                           table.seg_nc, seg_flags, partial, norms, float(lr), float(momentum),
                           float(weight_decay), float(eta), float(gscale), float(eps), bool(first),
                           dyn, skip)
        return
    if _skipped(skip):
        return
    flags = seg_flags.tolist()
    for i, (off, n) in enumerate(zip(table.seg_offsets, table.seg_sizes)):
        sl = slice(off, off + n)
        wi, gi = w[sl], g[sl].float() * gscale
        skip = flags[i] & 1
        wd = 0.0 if skip else weight_decay
        wn, gn = float(wi.norm()), float(gi.norm())
        trust = 1.0
        if not skip and wn > 0 and gn > 0:
            trust = eta * wn / (gn + wd * wn + eps)
        d = lr * trust * (gi + wd * wi)
        if first:
            mom[sl].copy_(d)
        else:
            mom[sl].mul_(momentum).add_(d)
        wi.sub_(mom[sl])
        if model is not None:
            model[sl].copy_(wi)


def seg_dot3(a: torch.Tensor, b: torch.Tensor, table: ChunkTable,
             workspace: Optional[dict] = None) -> torch.Tensor:
    """Per segment (a.b, |a|^2, |b|^2) as a [nseg, 3] fp32 tensor (deterministic).
    ``a`` may be fp32 while ``b`` is the (fp16/bf16) wire copy."""
    _check_table(table, min(a.numel(), b.numel()))
    if _on_gpu(a):
        ws = workspace if workspace is not None else {}
        partial = ws.get("partial3")
        if partial is None or partial.numel() < 3 * table.nchunks:
            partial = ws["partial3"] = torch.empty(3 * table.nchunks, dtype=torch.float32,
                                                   device=a.device)
        out = torch.empty(3 * table.nseg, dtype=torch.float32, device=a.device)
        native().seg_dot3(a, b, table.begin, table.len, table.seg, table.seg_c0, table.seg_nc,
                          partial, out)
        return out.view(-1, 3)
    rows = []
    for off, n in zip(table.seg_offsets, table.seg_sizes):
        x, y = a[off:off + n].float(), b[off:off + n].float()
        rows.append(torch.stack([(x * y).sum(), (x * x).sum(), (y * y).sum()]))
    return torch.stack(rows) if rows else torch.zeros(0, 3)


def adasum_combine(a: torch.Tensor, b: torch.Tensor, table: ChunkTable, dots: torch.Tensor) -> None:
    """a <- (1 - d/(2|a|^2)) a + (1 - d/(2|b|^2)) b per segment."""
    _check_table(table, min(a.numel(), b.numel()))
    if _on_gpu(a):
        native().adasum_combine(a, b, table.begin, table.len, table.seg, table.seg_c0,
                                table.seg_nc, dots.reshape(-1).contiguous())
        return
    d = dots.reshape(-1, 3).tolist()
    for i, (off, n) in enumerate(zip(table.seg_offsets, table.seg_sizes)):
        dot, na, nb = d[i]
        ca = 1.0 - dot / (2 * na) if na >= 1e-8 else 1.0
        cb = 1.0 - dot / (2 * nb) if nb >= 1e-8 else 1.0
        x = a[off:off + n]
        x.copy_(ca * x.float() + cb * b[off:off + n].float())


def adasum_fcombine(f: torch.Tensor, r: torch.Tensor, table: ChunkTable, dots: torch.Tensor,
                    swap: bool) -> None:
    """Vector-halving Adasum merge on the fp32 running sum ``f`` with the received
    (wire-dtype) copy ``r``: ``dots`` rows are (a.b, |a|^2, |b|^2) with a = the
    lower rank group's vector; ``swap`` means ``f`` holds b.  f <- ca*a + cb*b."""
    _check_table(table, min(f.numel(), r.numel()))
    if _on_gpu(f):
        native().adasum_fcombine(f, r, table.begin, table.len, table.seg, table.seg_c0,
                                 table.seg_nc, dots.reshape(-1).contiguous(), bool(swap))
        return
    d = dots.reshape(-1, 3).tolist()
    for i, (off, n) in enumerate(zip(table.seg_offsets, table.seg_sizes)):
        if n <= 0:
            continue
        dot, na, nb = d[i]
        ca = 1.0 - dot / (2 * na) if na >= 1e-8 else 1.0
        cb = 1.0 - dot / (2 * nb) if nb >= 1e-8 else 1.0
        cf, cr = (cb, ca) if swap else (ca, cb)
        x = f[off:off + n]
        x.copy_(cf * x + cr * r[off:off + n].float())


def tensor_from_ptr(ptr: int, numel: int, dtype: torch.dtype, device) -> torch.Tensor:
    """A 1-D tensor over device memory mivod owns elsewhere (the xGMI mesh's
    IPC staging slot) — no copy; the owner must outlive the view."""
    dev = torch.device(device)
    return native().tensor_from_ptr(int(ptr), int(numel), dtype, dev.index or 0)
