"""``mivod.torch.DistributedOptimizer`` — the PyTorch-ROCm hook path.

Parity: horovod 0.18.1 ``horovod/torch/__init__.py`` ``_DistributedOptimizer``
(SURVEY.md §2.2 U22): wraps any ``torch.optim.Optimizer``; gradients are
averaged across ranks as backward produces them; ``step()`` waits for the
reductions then applies the update; ``synchronize()``, ``skip_synchronize()``,
``backward_passes_per_step``, ``compression``, ``op`` (Average / Sum / Adasum),
duplicate-name checks, and the "zero_grad before synchronize" assertion.
The reference reaches the same behaviour through Keras
(/root/reference/mnist_keras.py:86-87, tensorflow2_keras_mnist.py:57-58).

MI355X design (not a translation of horovod's per-tensor async ops):

* **Static schedule.**  Buckets are planned once from the parameter layout —
  backward order, per dtype, ``MIVOD_FIRST_BUCKET_MB`` for the first bucket
  (the last layers, to start xGMI traffic early), ``MIVOD_BUCKET_MB`` after —
  and issued in the same order on every rank, so no per-step negotiation.
* **One pack launch per bucket.**  ``register_post_accumulate_grad_hook``
  marks a parameter ready; when its bucket is complete the hand-written
  multi-tensor pack kernel (K1, fused cast = compression, fused prescale) copies
  all its grads into the flat bucket on the compute stream.
* **Comm stream.**  The high-priority HIP comm stream waits on the pack event,
  runs the RCCL allreduce (xGMI ring), and — when the wrapped optimizer is a
  ``mivod.optim.Fused*`` — immediately runs the fused optimizer kernel (K6)
  on the reduced bucket with the 1/N average folded into its grad scale.  The
  whole update overlaps the remaining backward; ``step()`` is then only a
  stream wait.  Plain torch optimizers get zero-copy gradient views into the
  reduced bucket instead.
* **Overflow guard** (default with fp16 wire compression): after each bucket's
  collective a read-only scan kernel checks the REDUCED bucket — a non-finite
  contribution of any rank (bf16 gradients above the fp16 range included) or an
  fp16 overflow inside the reduction is non-finite there, with the same bits on
  every rank, so every rank sets the same device flag with no extra collective
  and no host sync.  Default ``MIVOD_GUARD_MODE=bucket``: the bucket's fused
  update runs immediately (overlapped with the rest of backward) and skips
  itself when its bucket is non-finite — the other buckets of that step are
  applied; an arena whose every bucket was skipped does not count the step.
  ``MIVOD_GUARD_MODE=step``: one flag per step and every update deferred to
  after the last bucket (horovod / AMP whole-step skip, not overlapped).  ``grad_scale="dynamic"`` additionally
  scales the wire by s (halved after an overflow, doubled back after
  ``MIVOD_GUARD_GROWTH_STEPS`` clean steps, capped at 1) and folds 1/s into the
  update.
* **Timeline**: with ``HOROVOD_TIMELINE`` set, every bucket's pack / collective
  / fused step is recorded with GPU timestamps (``utils.timeline.PhaseRecorder``).
"""
from __future__ import annotations

import contextlib
import threading
import warnings
from typing import Dict, List, Optional

import torch

from ..common import basics
from ..ops import kernels as K
from ..ops.compression import Compression
from ..optim.fused import Arena, FusedOptimizer, _align
from ..parallel import collectives as C
from ..parallel.order import ORDER
from ..utils import markers as MK
from ..utils import timeline as TL

_log = __import__("logging").getLogger("mivod")


class _GradArena:
    """Gradient-only arena for plain (non-fused) optimizers."""

    def __init__(self, params: List[torch.nn.Parameter], wire_dtype: torch.dtype):
        self.params = params
        self.offsets, o = [], 0
        for p in params:
            self.offsets.append(o)
            o += _align(p.numel())
        self.numel = o
        self.dtype = params[0].dtype
        self.grad_dtype = wire_dtype
        self.device = params[0].device
        self.grad = torch.zeros(o, dtype=wire_dtype, device=self.device)
        self.tables: Dict[tuple, K.ChunkTable] = {}

    def range_of(self, i0, i1):
        lo = self.offsets[i0]
        hi = self.offsets[i1] if i1 < len(self.params) else self.numel
        return lo, hi

    def slot(self, flat, i):
        p = self.params[i]
        return torch.as_strided(flat, p.size(), p.stride(), self.offsets[i])

    def table(self, i0, i1):
        key = (i0, i1)
        t = self.tables.get(key)
        if t is None:
            lo = self.offsets[i0]
            t = K.make_chunk_table([self.params[i].numel() for i in range(i0, i1)], self.device,
                                   [self.offsets[i] - lo for i in range(i0, i1)])
            self.tables[key] = t
        return t


class _Bucket:
    __slots__ = ("index", "arena", "i0", "i1", "lo", "hi", "params", "pending", "launched",
                 "order_key", "name")

    def __init__(self, index, arena, i0, i1, order_key):
        self.index = index
        self.arena = arena
        self.i0, self.i1 = i0, i1
        self.lo, self.hi = arena.range_of(i0, i1)
        self.params = arena.params[i0:i1]
        self.pending = len(self.params)
        self.launched = False
        self.order_key = order_key
        self.name = f"bucket.{index}"

    @property
    def nbytes(self):
        return (self.hi - self.lo) * self.arena.grad.element_size()


def plan_buckets(arenas, first_bucket_bytes: int, bucket_bytes: int, position,
                 last_bucket_bytes: int = 0) -> List[_Bucket]:
    """Split every arena (params in backward order) into contiguous buckets.

    The first bucket of the whole model (earliest in backward) is capped at
    ``first_bucket_bytes`` so xGMI traffic starts early; the last one (the
    first layers, whose gradients arrive when backward is already over) at
    ``last_bucket_bytes`` so the exposed tail — its allreduce + fused step after
    the final backward kernel — stays short; the rest at ``bucket_bytes``.
    Buckets are ordered by readiness (backward position of their last
    parameter), identically on all ranks.
    """
    raw = []
    for a in arenas:
        es = a.grad.element_size()
        i0 = 0
        cur = 0
        for i, p in enumerate(a.params):
            sz = _align(p.numel()) * es
            if cur > 0 and cur + sz > bucket_bytes:
                raw.append((a, i0, i))
                i0, cur = i, 0
            cur += sz
        raw.append((a, i0, len(a.params)))

    def key(r):
        # a bucket is ready when its LAST gradient arrives: order (and launch)
        # buckets by that, or a bucket holding one early-layer tensor (e.g. the
        # stem BatchNorm in the fp32 arena) would block every later launch
        return max(position[id(p)] for p in r[0].params[r[1]:r[2]])

    def split(r, cap, from_end):
        a, i0, i1 = r
        es = a.grad.element_size()
        rng = range(i1 - 1, i0 - 1, -1) if from_end else range(i0, i1)
        cur = 0
        for i in rng:
            cur += _align(a.params[i].numel()) * es
            if cur >= cap:
                cut = i if from_end else i + 1
                if i0 < cut < i1:
                    return [(a, i0, cut), (a, cut, i1)]
                return [r]
        return [r]

    raw.sort(key=key)
    if raw and first_bucket_bytes > 0:
        raw[0:1] = split(raw[0], first_bucket_bytes, False)
    raw.sort(key=key)
    if len(raw) > 1 and last_bucket_bytes > 0:
        raw[-1:] = split(raw[-1], last_bucket_bytes, True)
    raw.sort(key=key)
    return [_Bucket(k, a, i0, i1, key((a, i0, i1))) for k, (a, i0, i1) in enumerate(raw)]


class _DistributedOptimizerMixin:
    """Methods mixed in front of the wrapped optimizer's class."""

    # ------------------------------------------------------------------ setup
    def _mvd_setup(self, named_parameters, compression, backward_passes_per_step, op,
                   bucket_mb, first_bucket_mb, gradient_predivide_factor,
                   overflow_guard=None, grad_scale=None):
        st = basics.state()
        if not st.initialized:
            raise ValueError(basics._NOT_INIT)
        cfg = st.config
        if compression is None:
            compression = Compression.by_name(cfg.compression)   # MIVOD_COMPRESSION
        self._mvd_size = st.size
        # collectives run when there are peers, or on the 1-rank RCCL comm that
        # MIVOD_FORCE_COLLECTIVES=1 builds (exercises the GPU path on one GPU)
        self._mvd_comm = st.size > 1 or st.gpu is not None
        self._mvd_rank = st.rank
        self._mvd_compression = compression
        self._mvd_bpps = int(backward_passes_per_step)
        self._mvd_op = op
        self._mvd_predivide = float(gradient_predivide_factor)
        if op == C.Adasum and self._mvd_predivide != 1.0:
            raise ValueError("gradient_predivide_factor not supported with op == Adasum")
        self._mvd_lock = threading.RLock()

        all_params = [p for g in self.param_groups for p in g["params"]]
        if named_parameters is not None:
            named_parameters = list(named_parameters)
            if any(not isinstance(t, tuple) or len(t) != 2 for t in named_parameters):
                raise ValueError("named_parameters should be a sequence of tuples (name, parameter), "
                                 "usually produced by model.named_parameters().")
            names = [n for n, _ in named_parameters]
            dups = sorted({n for n in names if names.count(n) > 1})
            if dups:
                raise ValueError("Parameter names in named_parameters must be unique. Found "
                                 f"duplicates: {', '.join(dups)}")
            known = {id(p) for _, p in named_parameters}
            unnamed = [p for p in all_params if id(p) not in known]
            if unnamed:
                raise ValueError("named_parameters was specified, but one or more model "
                                 "parameters were not named. Python object ids: "
                                 f"{', '.join(str(id(p)) for p in unnamed)}")
            self._mvd_names = {id(p): n for n, p in named_parameters}
        else:
            self._mvd_names = {id(p): f"allreduce.noname.{i}" for i, p in enumerate(all_params)}

        trainable = [p for p in all_params if p.requires_grad]
        # backward position: reverse registration order
        self._mvd_position = {id(p): i for i, p in enumerate(reversed(trainable))}
        self._mvd_fused = isinstance(self, FusedOptimizer)
        wire = compression.wire_dtype
        if self._mvd_fused:
            self._mv_external_grads = True
            arenas = self._mv_build(grad_dtype_for=wire)
        else:
            arenas = []
            seen = set()
            by_key: Dict[tuple, List[torch.nn.Parameter]] = {}
            for p in reversed(trainable):
                if id(p) in seen:
                    continue
                seen.add(id(p))
                by_key.setdefault((p.dtype, p.device), []).append(p)
            for (dt, _dev), ps in by_key.items():
                arenas.append(_GradArena(ps, wire(dt)))
        self._mvd_arenas = arenas
        bmb = cfg.bucket_mb if bucket_mb is None else bucket_mb
        fmb = cfg.first_bucket_mb if first_bucket_mb is None else first_bucket_mb
        self._mvd_last_bytes = int(cfg.last_bucket_mb * 2 ** 20)
        self._mvd_buckets = plan_buckets(arenas, int(fmb * 2 ** 20), int(bmb * 2 ** 20),
                                         self._mvd_position, self._mvd_last_bytes)
        self._mvd_where: Dict[int, tuple] = {}
        for b in self._mvd_buckets:
            for k, p in enumerate(b.params):
                self._mvd_where[id(p)] = (b, b.i0 + k)
        self._mvd_counts: Dict[int, int] = {}
        self._mvd_next = 0
        self._mvd_in_step = False
        self._mvd_synchronized = False
        self._mvd_should_sync = True
        self._mvd_stream = st.comm_stream
        self._mvd_inline = False          # run comm + fused update on the current stream
        self._mvd_done_event = None
        self._mvd_nonfinite = None
        self._mvd_steps = 0
        # overflow guard (fp16 wire by default; MIVOD_OVERFLOW_GUARD=0/1 overrides)
        import os
        env_guard = os.environ.get("MIVOD_OVERFLOW_GUARD", "")
        if overflow_guard is None:
            overflow_guard = (env_guard == "1") if env_guard else (wire(torch.bfloat16)
                                                                     == torch.float16)
        self._mvd_guard = bool(overflow_guard) and self._mvd_fused
        if bool(overflow_guard) and not self._mvd_fused:
            warnings.warn("mivod overflow guard needs a mivod.optim.Fused* optimizer; disabled")
        self._mvd_dynamic = self._mvd_guard and (grad_scale == "dynamic" or
                                                 os.environ.get("MIVOD_GRAD_SCALE", "") ==
                                                 "dynamic")
        self._mvd_gs = float(grad_scale) if isinstance(grad_scale, (int, float)) else 1.0
        self._mvd_gs_growth = int(os.environ.get("MIVOD_GUARD_GROWTH_STEPS", "200"))
        self._mvd_gs_good = 0
        # "bucket" (default): each reduced bucket is scanned and its fused update
        # runs right away, skipped on every rank when that bucket is non-finite
        # (overlapped with backward); "step": one flag for the whole step, every
        # update deferred until the last bucket is reduced (horovod / AMP
        # whole-step semantics, not overlapped)
        self._mvd_guard_mode = os.environ.get("MIVOD_GUARD_MODE", "bucket")
        if self._mvd_guard_mode not in ("bucket", "step"):
            raise ValueError("MIVOD_GUARD_MODE must be 'bucket' or 'step'")
        self._mvd_flag = None             # device int32 non-finite flags of the step
        self._mvd_flag_host = None        # pinned copy + event of the previous step's flags
        self._mvd_flag_ev = None
        self._mvd_flag_plan = None        # the bucket plan those flags index
        self._mvd_skipped = 0
        self._mvd_rec = None
        self._mvd_comm_log = None         # time_comm(): [(bucket, bytes, ev0, ev1)]
        self._mvd_autotune = None
        if cfg.autotune and bucket_mb is None and first_bucket_mb is None:
            from ..parallel.autotune import BucketAutotuner
            self._mvd_autotune = BucketAutotuner(log_path=cfg.autotune_log)
            f0, b0 = self._mvd_autotune.current()
            self._mvd_replan(f0, b0)
        if st.size > 1:
            self._mvd_check_schedule()
        self._mvd_hooks = []
        for p in trainable:
            self._mvd_hooks.append(p.register_post_accumulate_grad_hook(self._mvd_hook))
        TL.note_plan(self._mvd_buckets)

    def _mvd_check_schedule(self):
        """Every rank must issue the same collectives in the same order: compare a
        64-bit hash of the static bucket plan (names, element counts, dtypes, op,
        compression) across ranks once, and raise on ALL ranks if they differ —
        instead of mismatched RCCL calls hanging or silently mixing tensors."""
        import hashlib
        h = hashlib.blake2b(digest_size=8)
        h.update(repr((C.op_name(self._mvd_op), self._mvd_compression.__name__,
                       self._mvd_bpps, self._mvd_guard, self._mvd_gs,
                       self._mvd_guard_mode if self._mvd_guard else "")).encode())
        for b in self._mvd_buckets:
            h.update(repr((str(b.arena.grad.dtype), b.hi - b.lo,
                           [(self._mvd_names[id(p)], tuple(p.shape)) for p in b.params])).encode())
        v = int.from_bytes(h.digest(), "little", signed=True)
        every = C.allgather(torch.tensor([v], dtype=torch.int64))   # CPU: native ring / gloo
        if not bool((every == every[0]).all()):
            raise ValueError(
                "mivod DistributedOptimizer: the static gradient schedule differs across ranks "
                f"(plan hashes {sorted(set(every.tolist()))}); every rank must wrap the same "
                "model with the same parameter order, dtypes, op, compression and bucket settings")

    # --------------------------------------------------------------- hot path
    def _mvd_hook(self, p: torch.Tensor):
        with self._mvd_lock:
            c = self._mvd_counts.get(id(p), 0) + 1
            self._mvd_counts[id(p)] = c
            if c < self._mvd_bpps:
                return
            if c > self._mvd_bpps:
                raise AssertionError(
                    "Gradients were computed more than backward_passes_per_step times before call "
                    "to step(). Increase backward_passes_per_step to accumulate gradients locally.")
            b, _ = self._mvd_where[id(p)]
            b.pending -= 1
            if b.pending == 0 and not self._mvd_inline:
                self._mvd_launch_ready()

    def _mvd_launch_ready(self):
        bs = self._mvd_buckets
        while self._mvd_next < len(bs) and bs[self._mvd_next].pending == 0:
            self._mvd_launch(bs[self._mvd_next])
            self._mvd_next += 1

    def _mvd_resolve_flags(self):
        """Consume the previous step's overflow flags (host wait on an event
        recorded after that step's last fused update — long done by the time the
        next step starts): skipped-step count, optimizer step counters, dynamic
        wire scale.  Every rank reads the same flags (they come from the reduced
        buckets), so every rank takes the same decisions."""
        if self._mvd_flag_ev is None:
            return
        self._mvd_flag_ev.synchronize()
        flags = [int(v) for v in self._mvd_flag_host.tolist()]
        plan = self._mvd_flag_plan or []
        self._mvd_flag_ev = None
        self._mvd_flag_plan = None
        if any(flags):
            self._mvd_skipped += 1
            if self._mvd_guard_mode == "step":
                skipped = list(plan)
                what = f"optimizer step {self._mvd_steps} skipped on every rank"
            else:
                skipped = [b for b in plan if flags[b.index]]
                what = (f"{len(skipped)} of {len(plan)} gradient buckets of optimizer step "
                        f"{self._mvd_steps} skipped on every rank ("
                        + ", ".join(b.name for b in skipped) + ")")
            if self._mvd_fused:
                for a in self._mvd_arenas:
                    mine = [b for b in plan if b.arena is a]
                    if mine and all(b in skipped for b in mine):
                        a.step = max(a.step - 1, 0)   # no update of this arena counted
            msg = f"mivod: non-finite gradients on the fp16 wire (or in the gradients) — {what}"
            if self._mvd_dynamic:
                self._mvd_gs = max(self._mvd_gs * 0.5, 2.0 ** -24)
                msg += f"; wire scale -> {self._mvd_gs:g}"
                self._mvd_gs_good = 0
            _log.warning(msg)
            warnings.warn(msg)
        elif self._mvd_dynamic:
            self._mvd_gs_good += 1
            if self._mvd_gs_good >= self._mvd_gs_growth and self._mvd_gs < 1.0:
                self._mvd_gs = min(self._mvd_gs * 2.0, 1.0)
                self._mvd_gs_good = 0

    def _mvd_guard_begin(self, device):
        """Step start (guard on): consume the previous step's flags, then reset."""
        self._mvd_resolve_flags()
        nf = len(self._mvd_buckets) if self._mvd_guard_mode == "bucket" else 1
        if self._mvd_flag is None or self._mvd_flag.numel() != nf:
            self._mvd_flag = torch.zeros(nf, dtype=torch.int32, device=device)
            self._mvd_flag_host = torch.zeros(nf, dtype=torch.int32)
            if device.type == "cuda":
                self._mvd_flag_host = self._mvd_flag_host.pin_memory()
        else:
            self._mvd_flag.zero_()

    def _mvd_bucket_flag(self, b: _Bucket):
        """The device flag a bucket's scan sets and its fused update reads."""
        if self._mvd_guard_mode == "bucket":
            return self._mvd_flag[b.index:b.index + 1]
        return self._mvd_flag[0:1]

    def state_dict(self):
        # a step skipped by the overflow guard must not be counted in the saved
        # optimizer state (its flags are otherwise read at the next step's start)
        if getattr(self, "_mvd_guard", False):
            self._mvd_resolve_flags()
        return super().state_dict()

    def _mvd_mesh_for(self, flat: torch.Tensor, cuda: bool, inplace: bool):
        """The xGMI mesh transport when this bucket rides it (pack straight into
        the mesh's IPC staging slot), else None."""
        st = basics.state()
        mesh = st.mesh
        if (mesh is None or not cuda or not self._mvd_comm or inplace
                or self._mvd_op == C.Adasum):
            return None
        return mesh if mesh.accepts(flat, "sum") else None

    def _mvd_launch(self, b: _Bucket):
        a = b.arena
        if not self._mvd_in_step:
            self._mvd_in_step = True
            self._mvd_rec = TL.recorder()
            if self._mvd_guard:
                self._mvd_guard_begin(a.grad.device)
            if self._mvd_fused:
                self._mv_begin_step()
        size = self._mvd_size
        prescale = 1.0 / self._mvd_predivide if self._mvd_op == C.Average else 1.0
        prescale *= self._mvd_gs
        rec = self._mvd_rec
        t_pack = rec.event() if rec is not None and a.grad.is_cuda else (
            rec.host() if rec is not None else None)
        groups: Dict[torch.dtype, tuple] = {}
        missing = []
        inplace = False
        with torch.no_grad():
            for k, p in enumerate(b.params):
                i = b.i0 + k
                g = p.grad
                lo = a.offsets[i]
                if g is None:
                    missing.append((lo, p.numel()))
                    continue
                if g.is_sparse:
                    g = g.to_dense()          # sparse_as_dense (embedding grads)
                if g.data_ptr() == a.grad.data_ptr() + lo * a.grad.element_size() and \
                        g.dtype == a.grad.dtype and g.stride() == p.stride():
                    if prescale != 1.0:
                        g.mul_(prescale)
                    inplace = True
                    continue  # gradient already lives in its bucket slot (accumulated in place)
                if g.stride() != p.stride() or not K.is_dense(g):
                    g = torch.empty_like(p, dtype=g.dtype).copy_(g)
                ent = groups.setdefault(g.dtype, ([], []))
                ent[0].append(g)
                ent[1].append(lo)
        flat = a.grad[b.lo:b.hi]
        # inline (no comm-stream fork; launched from synchronize(), after backward) while
        # a single-rank step is captured into a HIP graph: ROCm runs a two-stream graph
        # DAG ~15 us/kernel slower than one chain (scripts/debug/graph_speed.py), and
        # with one rank there is no RCCL to overlap
        cuda = flat.is_cuda and self._mvd_stream is not None and not self._mvd_inline
        mesh = self._mvd_mesh_for(flat, cuda, inplace)
        # the mesh's staging slot is chosen by its call count, so pack + collective
        # are ONE entry of the cross-rank issue order (no collective in between)
        order = ORDER.issue() if mesh is not None else contextlib.nullcontext()
        with order:
            with torch.no_grad():
                if mesh is not None:
                    dst, base = mesh.stage_view(flat.numel(), flat.dtype), b.lo
                else:
                    dst, base = a.grad, 0
                for lo, n in missing:
                    dst[lo - base:lo - base + n].zero_()
                with MK.range(f"mivod.pack.{b.name}"):
                    for dt, (gl, ol) in groups.items():
                        K.pack(gl, dst, [o - base for o in ol], scale=prescale)
                if self._mvd_fused:
                    for p in b.params:
                        p.grad = None            # freed on the compute stream after the pack
            t_packed = None
            if rec is not None:
                t_packed = rec.event() if flat.is_cuda else rec.host()
                rec.add(b.name, "MEMCPY_IN_FUSION_BUFFER", t_pack, t_packed)
            if cuda:
                ev = torch.cuda.Event()
                ev.record()
                ctx = torch.cuda.stream(self._mvd_stream)
            else:
                ctx = contextlib.nullcontext()
            with ctx:
                if cuda:
                    self._mvd_stream.wait_event(ev)
                if self._mvd_comm:
                    t0 = (rec.event() if cuda else rec.host()) if rec is not None else None
                    c0 = self._mvd_comm_event() if cuda else None
                    with MK.range(f"mivod.allreduce.{b.name}"):
                        if mesh is not None:
                            avg = self._mvd_op == C.Average and not self._mvd_fused
                            mesh.allreduce_into(flat, dst, "avg" if avg else "sum")
                        elif self._mvd_op == C.Adasum:
                            C.allreduce_(flat, C.Adasum, adasum_table=a.table(b.i0, b.i1))
                        elif self._mvd_fused:
                            C.allreduce_(flat, C.Sum)
                        else:
                            C.allreduce_(flat, C.Average if self._mvd_op == C.Average else C.Sum)
                    if c0 is not None:
                        self._mvd_comm_log.append((b.name, b.nbytes, c0, self._mvd_comm_event()))
                    if rec is not None:
                        phase = "ADASUM" if self._mvd_op == C.Adasum else (
                            "MESH_ALLREDUCE" if mesh is not None else (
                                "NCCL_ALLREDUCE" if cuda else "RING_ALLREDUCE"))
                        rec.add(b.name, phase, t0, rec.event() if cuda else rec.host())
        with (torch.cuda.stream(self._mvd_stream) if cuda else contextlib.nullcontext()):
            if self._mvd_guard:
                # overflow guard: scan the REDUCED bucket (a non-finite contribution
                # of any rank, or an fp16 overflow in the reduction, is non-finite
                # here, identically on every rank — no extra collective)
                K.nonfinite_scan(flat, self._mvd_bucket_flag(b))
            if self._mvd_fused:
                if not self._mvd_guard or self._mvd_guard_mode == "bucket":
                    self._mvd_apply_bucket(b, cuda)
            else:
                post = self._mvd_predivide if (self._mvd_op == C.Average and size > 1) else 1.0
                t0 = (rec.event() if cuda else rec.host()) if rec is not None else None
                if post != 1.0:
                    flat.mul_(post)
                self._mvd_expose_grads(b)
                if rec is not None:
                    rec.add(b.name, "MEMCPY_OUT_FUSION_BUFFER", t0,
                            rec.event() if cuda else rec.host())
            if cuda:
                ev2 = torch.cuda.Event()
                ev2.record()
                self._mvd_done_event = ev2
        b.launched = True

    # ------------------------------------------------------- comm timing
    def _mvd_comm_event(self):
        if self._mvd_comm_log is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def time_comm(self, enable: bool = True):
        """Record a timing-event pair around every bucket collective (on the comm
        stream) from now on — bench.py's measured per-bucket allreduce time and
        bus bandwidth.  ``comm_timings()`` reads and clears them."""
        self._mvd_comm_log = [] if enable else None

    def comm_timings(self) -> List[tuple]:
        """[(bucket name, payload bytes, ms)] of every collective recorded since
        ``time_comm()`` / the last call (waits for them to finish)."""
        log = self._mvd_comm_log or []
        out = []
        for name, nb, e0, e1 in log:
            e1.synchronize()
            out.append((name, nb, e0.elapsed_time(e1)))
        if self._mvd_comm_log is not None:
            self._mvd_comm_log = []
        return out

    def _mvd_apply_bucket(self, b: _Bucket, cuda: bool):
        """The fused optimizer step of one reduced bucket (current stream)."""
        rec = self._mvd_rec
        gscale = 1.0 / self._mvd_gs
        if self._mvd_op == C.Average:
            gscale *= self._mvd_predivide / self._mvd_size
        t0 = (rec.event() if cuda else rec.host()) if rec is not None else None
        self._mv_skip = self._mvd_bucket_flag(b) if self._mvd_guard else None
        with MK.range(f"mivod.step.{b.name}"):
            self._mv_apply(b.arena, b.i0, b.i1, gscale)
        self._mv_skip = None
        if rec is not None:
            rec.add(b.name, "OPTIMIZER_STEP", t0, rec.event() if cuda else rec.host())

    def _mvd_guard_finish(self):
        """synchronize() with the guard on, after the last bucket: ("step" mode)
        run every bucket's fused update with the step's flag; then copy the flags
        to pinned host memory for the next step's bookkeeping."""
        flag = self._mvd_flag
        if flag is None:
            return
        cuda = flag.is_cuda and self._mvd_stream is not None and not self._mvd_inline
        ctx = torch.cuda.stream(self._mvd_stream) if cuda else contextlib.nullcontext()
        with ctx:
            if self._mvd_guard_mode == "step":
                for b in self._mvd_buckets:
                    self._mvd_apply_bucket(b, cuda)
            self._mvd_flag_plan = list(self._mvd_buckets)
            if flag.is_cuda:
                self._mvd_flag_host.copy_(flag, non_blocking=True)
                self._mvd_flag_ev = torch.cuda.Event()
                self._mvd_flag_ev.record()
            else:
                self._mvd_flag_host.copy_(flag)
                self._mvd_flag_ev = _DoneEvent()
            if cuda:
                ev2 = torch.cuda.Event()
                ev2.record()
                self._mvd_done_event = ev2

    def guard_stats(self) -> dict:
        """Overflow-guard counters (skipped steps so far, current wire scale)."""
        return {"enabled": self._mvd_guard, "mode": self._mvd_guard_mode,
                "skipped_steps": self._mvd_skipped,
                "wire_scale": self._mvd_gs, "dynamic": self._mvd_dynamic}

    def _mvd_expose_grads(self, b: _Bucket):
        """Plain optimizers: p.grad := reduced values (zero-copy view when the
        wire dtype equals the grad dtype, fused unpack + decompress otherwise)."""
        a = b.arena
        same = a.grad.dtype == a.dtype
        if same:
            for k, p in enumerate(b.params):
                p.grad = a.slot(a.grad, b.i0 + k)
            return
        outs, offs = [], []
        for k, p in enumerate(b.params):
            i = b.i0 + k
            if p.grad is None or p.grad.dtype != p.dtype or p.grad.stride() != p.stride():
                p.grad = torch.empty_like(p)
            outs.append(p.grad)
            offs.append(a.offsets[i])
        K.unpack(outs, a.grad, offs)

    # -------------------------------------------------------------- user API
    def synchronize(self):
        with self._mvd_lock:
            # buckets not launched by the hooks (unused parameters, a partial
            # backward_passes_per_step window) reduce now, missing grads as zeros
            for b in self._mvd_buckets:
                if not b.launched:
                    b.pending = 0
            self._mvd_launch_ready()
            if self._mvd_guard and self._mvd_in_step:
                self._mvd_guard_finish()
            if self._mvd_stream is not None and torch.cuda.is_available() and \
                    not self._mvd_inline:
                torch.cuda.current_stream().wait_stream(self._mvd_stream)
            if self._mvd_fused:
                self._mv_end_step()
            for b in self._mvd_buckets:
                b.launched = False
                b.pending = len(b.params)
            self._mvd_counts.clear()
            self._mvd_next = 0
            self._mvd_in_step = False
            self._mvd_synchronized = True
            self._mvd_steps += 1
            if self._mvd_autotune is not None and not self._mvd_autotune.done:
                self._mvd_autotune_step()
        from ..utils import faults
        faults.maybe_inject(self._mvd_rank, self._mvd_steps)

    def _mvd_replan(self, first_mb: float, bucket_mb: float):
        self._mvd_buckets = plan_buckets(self._mvd_arenas, int(first_mb * 2 ** 20),
                                         int(bucket_mb * 2 ** 20), self._mvd_position,
                                         self._mvd_last_bytes)
        self._mvd_where = {}
        for b in self._mvd_buckets:
            for k, p in enumerate(b.params):
                self._mvd_where[id(p)] = (b, b.i0 + k)

    def _mvd_autotune_step(self):
        def sync():
            if self._mvd_stream is not None:
                torch.cuda.synchronize()
        cand = self._mvd_autotune.on_step_end(sync)
        if cand is None:
            return
        if self._mvd_size > 1:           # everybody adopts rank 0's decision
            from .functions import broadcast_object
            cand = broadcast_object(cand, root_rank=0)
        self._mvd_replan(*cand)

    @contextlib.contextmanager
    def skip_synchronize(self):
        """Use after an explicit ``synchronize()`` (e.g. to clip gradients)."""
        self._mvd_should_sync = False
        try:
            yield
        finally:
            self._mvd_should_sync = True

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._mvd_should_sync:
            if self._mvd_synchronized:
                warnings.warn("optimizer.step() called without a loss.backward() since the last "
                              "synchronize(); re-using the last reduced gradients.")
            else:
                self.synchronize()
        elif not self._mvd_synchronized:
            raise AssertionError("skip_synchronize() used without a preceding synchronize()")
        self._mvd_synchronized = False
        if self._mvd_fused:
            return loss           # the fused update already ran on the comm stream
        super().step()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        if self._mvd_in_step:
            raise AssertionError("optimizer.zero_grad() was called after loss.backward() but before "
                                 "optimizer.step() or optimizer.synchronize(). This is prohibited "
                                 "as it can cause a race condition.")
        return super().zero_grad(set_to_none=set_to_none)

    def bucket_plan(self):
        """[(name, nbytes, [param names])] of the static schedule."""
        return [(b.name, b.nbytes, [self._mvd_names[id(p)] for p in b.params])
                for b in self._mvd_buckets]


class _DoneEvent:
    def synchronize(self):
        pass


def DistributedOptimizer(optimizer, named_parameters=None, compression=None,
                         backward_passes_per_step: int = 1, op=C.Average, bucket_mb=None,
                         first_bucket_mb=None, gradient_predivide_factor: float = 1.0,
                         overflow_guard=None, grad_scale=None):
    """Wrap ``optimizer`` so gradients are averaged (``op``) across all ranks.

    ``compression`` defaults to ``MIVOD_COMPRESSION`` (``none``).  With an fp16
    wire the overflow guard is on unless ``overflow_guard=False``;
    ``grad_scale="dynamic"`` (or a float) scales the wire (see module doc).

    Returns an instance of a dynamically created subclass of the optimizer's
    class (same class name, so ``isinstance`` and pickled configs keep working),
    carrying over the optimizer's state and param groups.
    """
    base = optimizer.__class__
    if isinstance(optimizer, _DistributedOptimizerMixin):
        raise ValueError("optimizer is already a mivod DistributedOptimizer")
    cls = type(base.__name__, (_DistributedOptimizerMixin, base), {"__module__": base.__module__})
    obj = cls.__new__(cls)
    obj.__dict__.update(optimizer.__dict__)
    obj._mvd_setup(named_parameters, compression, backward_passes_per_step, op, bucket_mb,
                   first_bucket_mb, gradient_predivide_factor, overflow_guard, grad_scale)
    return obj
