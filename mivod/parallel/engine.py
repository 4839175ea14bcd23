"""Named asynchronous collectives with cross-rank negotiation (the horovod
"background thread" model, SURVEY.md §2.2 U2–U7, U13, U15).

``allreduce_async(t, name=...)`` and friends enqueue a request and return a
handle immediately.  A background thread runs a cycle every
``HOROVOD_CYCLE_TIME`` ms (or as soon as work arrives): it hands the pending
requests to the *controller* — the C++ coordinator in ``mivod._mvcore`` over
TCP when size > 1 — which replies with the globally agreed, ordered and fused
list of responses (tensors submitted by every rank, validated for matching
dtype/shape/op/root, fused up to ``HOROVOD_FUSION_THRESHOLD``).  Every rank then
executes the identical response list, so the RCCL/gloo collectives match.

GPU execution happens on mivod's high-priority HIP comm stream — the same
stream and the same RCCL communicator as the static gradient schedule, in the
cross-rank order of ``order.ORDER`` (each cycle reports this rank's collective
count; the coordinator answers with the point at which the cycle's GPU
responses run): wait on each tensor's ready event, one multi-tensor pack kernel
(K1, fused compression cast + prescale) into the persistent fusion buffer, one
RCCL collective, one unpack kernel (K2, fused decompress + postscale), done
event.  The host never waits on the GPU; ``synchronize(handle)`` makes the
caller's stream wait on the done event.

The request a rank submits carries the *wire* dtype (after compression) and the
pre-/postscale factors, so the coordinator validates and fuses on what actually
travels (horovod compresses before enqueueing, which has the same effect).
"""
from __future__ import annotations

import itertools
import logging
import os
import threading
import time
from typing import Dict, List, Optional

import torch

from ..ops import kernels as K
from ..ops.compression import Compression
from . import collectives as C
from .order import ORDER

log = logging.getLogger("mivod")

ALLREDUCE, ALLGATHER, BROADCAST, ALLTOALL = 0, 1, 2, 3
KIND_NAMES = {ALLREDUCE: "allreduce", ALLGATHER: "allgather", BROADCAST: "broadcast",
              ALLTOALL: "alltoall"}
_DTYPE_CODE = {torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16",
               torch.float64: "f64", torch.int32: "i32", torch.int64: "i64", torch.uint8: "u8",
               torch.int8: "i8", torch.bool: "b1", torch.int16: "i16"}


class HorovodInternalError(RuntimeError):
    pass


class Handle:
    __slots__ = ("name", "kind", "tensor", "output", "op", "root", "compression", "ctx",
                 "prescale", "postscale", "ready_event", "done_event", "done", "error", "result",
                 "splits", "enqueue_time")

    def __init__(self, name, kind, tensor, output, op, root, compression, prescale, postscale,
                 splits=None):
        self.name = name
        self.kind = kind
        self.tensor = tensor
        self.output = output
        self.op = op
        self.root = root
        self.compression = compression
        self.ctx = None
        self.prescale = prescale
        self.postscale = postscale
        self.ready_event = None
        self.done_event = None
        self.done = threading.Event()
        self.error: Optional[BaseException] = None
        self.result = None
        self.splits = splits
        self.enqueue_time = time.time()

    def wire_dtype(self) -> torch.dtype:
        t = self.tensor
        if self.kind != ALLREDUCE or not t.dtype.is_floating_point:
            return t.dtype
        return self.compression.wire_dtype(t.dtype)

    def request(self, device_index: int):
        t = self.tensor
        wd = self.wire_dtype()
        es = torch.empty((), dtype=wd).element_size()
        return (self.name, self.kind, _DTYPE_CODE.get(wd, str(wd)), tuple(t.shape),
                int(self.root), int(self.op), device_index, t.numel() * es,
                float(self.prescale), float(self.postscale))


class LocalController:
    """size == 1: every request is immediately ready; fuse consecutive
    allreduces of one dtype/op up to the threshold (same rules as the C++
    coordinator)."""

    def __init__(self, fusion_threshold: int):
        self.fusion_threshold = fusion_threshold

    def negotiate(self, requests, shutdown=False, position=0):
        return (fuse_responses([(r[1], [r[0]], "") for r in requests],
                               {r[0]: r for r in requests}, self.fusion_threshold),
                shutdown, position)

    def close(self):
        pass


def fuse_responses(responses, req_by_name, threshold):
    out = []
    for kind, names, err in responses:
        if (out and not err and kind == ALLREDUCE and out[-1][0] == ALLREDUCE and not out[-1][2]):
            prev = out[-1][1]
            r0, r1 = req_by_name[prev[0]], req_by_name[names[0]]
            same = (r0[2] == r1[2] and r0[5] == r1[5] and (r0[6] < 0) == (r1[6] < 0)
                    and tuple(r0[8:10]) == tuple(r1[8:10]))
            total = sum(req_by_name[n][7] for n in prev) + r1[7]
            if same and total <= threshold and r1[5] != C.Adasum:
                prev.extend(names)
                continue
        out.append((kind, list(names), err))
    return out


class Engine:
    def __init__(self, state):
        self.st = state
        cfg = state.config
        self.cfg = cfg
        self.pending: List[Handle] = []
        self.inflight: Dict[str, Handle] = {}
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self.counter = itertools.count()
        self.thread: Optional[threading.Thread] = None
        self.running = False
        self.stream = None
        self.fusion: Dict[tuple, torch.Tensor] = {}
        self.controller = None
        self.loop = None
        self.native = False
        self.tl = None

    # ------------------------------------------------------------ lifecycle
    def start(self):
        st = self.st
        if st.device.type == "cuda":
            # ONE comm stream for the bucket schedule and the named ops
            self.stream = st.comm_stream or torch.cuda.Stream(device=st.device, priority=-1)
        from ..utils import timeline as TL
        self.tl = TL.get()
        self.native = os.environ.get("MIVOD_ENGINE", "native") != "python"
        if self.native:
            # negotiation cycle in a native thread (csrc/engine/loop.cc); this
            # process's Python only enqueues and executes responses
            from .controller import make_controller
            from .. import _mvcore  # type: ignore
            self.controller = make_controller(st, self.cfg)
            cycle = max(self.cfg.cycle_time_ms, 0.0) / 1000.0
            self.loop = _mvcore.EngineLoop(self.controller.ctl, st.size, cycle)
            ORDER.on_position = self.loop.set_position
            self.loop.set_position(ORDER.position())
            target = self._exec_loop
        else:
            if st.size == 1:
                self.controller = LocalController(self.cfg.fusion_threshold)
            else:
                from .controller import make_controller
                self.controller = make_controller(st, self.cfg)
            target = self._loop
        self.running = True
        self.thread = threading.Thread(target=target, name="mivod-engine", daemon=True)
        self.thread.start()

    def stop(self):
        if not self.running:
            return
        with self.cv:
            self.running = False
            self.cv.notify_all()
        if self.loop is not None:
            self.loop.request_shutdown()
        if self.thread is not None:
            self.thread.join(timeout=30)
        if self.loop is not None:
            if ORDER.on_position == self.loop.set_position:
                ORDER.on_position = None
            if self.loop.finished:
                self.loop.join()
        if self.controller is not None:
            self.controller.close()

    # -------------------------------------------------------------- enqueue
    def enqueue(self, kind, tensor, output=None, name=None, op=C.Average, root=0,
                compression=Compression.none, prescale=1.0, postscale=1.0, splits=None) -> Handle:
        if not self.running:
            raise ValueError("Horovod has not been initialized; use hvd.init().")
        if name is None:
            name = f"{KIND_NAMES[kind]}.noname.{next(self.counter)}"
        h = Handle(name, kind, tensor, output, op, root, compression, prescale, postscale, splits)
        if tensor.is_cuda:
            h.ready_event = torch.cuda.Event()
            h.ready_event.record()
        with self.cv:
            if name in self.inflight:
                raise ValueError(f"Duplicate name '{name}' submitted before the previous "
                                 "operation with that name completed")
            self.inflight[name] = h
            if tensor.is_cuda:
                ORDER.submitted(1)      # direct GPU collectives wait for its response
            if self.loop is None:
                self.pending.append(h)
                self.cv.notify_all()
        if self.tl is not None:
            self.tl.start(name, "QUEUE")
        if self.loop is not None:
            self.loop.submit([h.request(self.st.device.index if tensor.is_cuda else -1)])
        return h

    # ----------------------------------------------------------------- loop
    def _exec_loop(self):
        """Executor of the native loop's responses (GIL released while waiting)."""
        while True:
            r = self.loop.wait(1.0)
            if r is None:
                if self.loop.finished:
                    break
                continue
            responses, all_shutdown, exec_at, err = r
            if err:
                log.error("mivod negotiation failed: %s", err)
                self._fail_all(HorovodInternalError(err))
                break
            with self.cv:
                waiting = dict(self.inflight)
            self._dispatch(responses, exec_at, waiting)
            if all_shutdown:
                self._fail_all(HorovodInternalError("mivod shut down with pending operations"))
                break

    def _dispatch(self, responses, exec_at, waiting):
        gpu_fns, n_gpu = [], 0
        for kind, names, err in responses:
            hs = [waiting.pop(n) for n in names if n in waiting]
            if not hs:
                continue
            on_gpu = hs[0].tensor.is_cuda
            if on_gpu:
                n_gpu += len(hs)
            if err:
                for h in hs:
                    self._finish(h, error=HorovodInternalError(err))
                continue
            if on_gpu:
                gpu_fns.append(lambda kind=kind, hs=hs: self._run(kind, hs))
            else:
                self._run(kind, hs)
        if n_gpu:
            ORDER.responded(exec_at, n_gpu, gpu_fns)

    def _loop(self):
        cycle = max(self.cfg.cycle_time_ms, 0.0) / 1000.0
        self._waiting: Dict[str, Handle] = {}
        while True:
            with self.cv:
                if self.running and not self.pending:
                    self.cv.wait(timeout=cycle if self.st.size > 1 else None)
                batch = self.pending
                self.pending = []
                stopping = not self.running
            reqs = [h.request(self.st.device.index if h.tensor.is_cuda else -1) for h in batch]
            self._waiting.update({h.name: h for h in batch})
            position = ORDER.position()
            try:
                responses, all_shutdown, exec_at = self.controller.negotiate(reqs, stopping,
                                                                             position)
            except Exception as e:  # control plane failure: fail every outstanding op
                log.error("mivod negotiation failed: %s", e)
                self._fail_all(HorovodInternalError(str(e)))
                break
            self._dispatch(responses, exec_at, self._waiting)
            if stopping and all_shutdown:
                self._fail_all(HorovodInternalError("mivod shut down with pending operations"))
                break

    def _run(self, kind, hs: List[Handle]):
        try:
            self._execute(kind, hs)
        except Exception as e:
            log.exception("mivod collective failed")
            for h in hs:
                if not h.done.is_set():
                    self._finish(h, error=HorovodInternalError(repr(e)))

    def _fail_all(self, err):
        n_gpu = 0
        if self.loop is not None:
            with self.cv:
                self._waiting = dict(self.inflight)
        for h in list(self._waiting.values()):
            n_gpu += int(h.tensor.is_cuda)
            self._finish(h, error=err)
        self._waiting = {}
        with self.cv:
            for h in self.pending:
                n_gpu += int(h.tensor.is_cuda)
                self._finish(h, error=err)
            self.pending = []
        if n_gpu:
            ORDER.responded(ORDER.position(), n_gpu, [])

    def _finish(self, h: Handle, error=None):
        h.error = error
        with self.cv:
            self.inflight.pop(h.name, None)
        if self.tl is not None:
            self.tl.end(h.name)
        h.done.set()

    # -------------------------------------------------------------- execute
    def _execute(self, kind, hs: List[Handle]):
        cuda = hs[0].tensor.is_cuda and self.stream is not None
        if cuda:
            with torch.cuda.stream(self.stream):
                for h in hs:
                    self.stream.wait_event(h.ready_event)
                    # caller-stream allocations used on the comm stream
                    h.tensor.record_stream(self.stream)
                    if h.output is not None and h.output.data_ptr() != h.tensor.data_ptr():
                        h.output.record_stream(self.stream)
                self._execute_on_stream(kind, hs)
                for h in hs:
                    h.done_event = torch.cuda.Event()
                    h.done_event.record(self.stream)
        else:
            self._execute_on_stream(kind, hs)
        for h in hs:
            self._finish(h)

    def _fusion_buffer(self, dtype, device, numel):
        key = (dtype, str(device))
        buf = self.fusion.get(key)
        if buf is None or buf.numel() < numel:
            buf = torch.empty(max(numel, 1 << 20), dtype=dtype, device=device)
            self.fusion[key] = buf
        return buf[:numel]

    def _execute_on_stream(self, kind, hs: List[Handle]):
        tl = self.tl
        if kind == ALLREDUCE:
            h0 = hs[0]
            wire = h0.wire_dtype()
            if len(hs) == 1 and wire == h0.tensor.dtype and h0.prescale == 1.0 and \
                    h0.output is not None and h0.tensor.is_contiguous():
                out = h0.output
                if out.data_ptr() != h0.tensor.data_ptr():
                    out.copy_(h0.tensor)
                if tl: tl.activity(h0.name, _coll_phase(out))
                table = K.make_chunk_table([out.numel()], out.device) if h0.op == C.Adasum else None
                C.allreduce_(out.view(-1), h0.op, engine=True, adasum_table=table)
                if h0.postscale != 1.0:
                    out.mul_(h0.postscale)
                h0.result = out
                return
            total = 0
            offs = []
            for h in hs:
                offs.append(total)
                total += (h.tensor.numel() + 63) // 64 * 64
            dev = h0.tensor.device
            buf = self._fusion_buffer(wire, dev, total)
            if tl:
                for h in hs: tl.activity(h.name, "MEMCPY_IN_FUSION_BUFFER")
            float_path = h0.tensor.dtype in (torch.float32, torch.float16, torch.bfloat16)
            if float_path:
                # one pack launch per (dtype, prescale): every handle keeps its own factor
                by_key: Dict[tuple, tuple] = {}
                for h, o in zip(hs, offs):
                    t = h.tensor if h.tensor.is_contiguous() else h.tensor.contiguous()
                    e = by_key.setdefault((t.dtype, float(h.prescale)), ([], []))
                    e[0].append(t)
                    e[1].append(o)
                for (_dt, pre), (ts, os_) in by_key.items():
                    K.pack(ts, buf, os_, scale=pre)
            else:
                for h, o in zip(hs, offs):
                    v = h.tensor.reshape(-1)
                    buf[o:o + h.tensor.numel()].copy_(v * h.prescale if h.prescale != 1.0 else v)
            if tl:
                for h in hs: tl.activity(h.name, _coll_phase(buf))
            table = None
            if h0.op == C.Adasum:
                table = K.make_chunk_table([h.tensor.numel() for h in hs], dev, offs)
            C.allreduce_(buf, h0.op, engine=True, adasum_table=table)
            if tl:
                for h in hs: tl.activity(h.name, "MEMCPY_OUT_FUSION_BUFFER")
            for h, o in zip(hs, offs):
                out = h.output
                if out is None:
                    out = torch.empty_like(h.tensor, memory_format=torch.contiguous_format)
                if float_path and out.is_contiguous():
                    K.unpack([out], buf, [o], scale=h.postscale)
                else:
                    v = buf[o:o + h.tensor.numel()].view(h.tensor.shape)
                    out.copy_(v * h.postscale if h.postscale != 1.0 else v)
                h.result = out
        elif kind == ALLGATHER:
            for h in hs:
                if tl: tl.activity(h.name, "ALLGATHER")
                h.result = C.allgather(h.tensor, engine=True)
        elif kind == BROADCAST:
            for h in hs:
                if tl: tl.activity(h.name, "BROADCAST")
                out = h.output if h.output is not None else h.tensor.clone()
                if out.data_ptr() != h.tensor.data_ptr():
                    out.copy_(h.tensor)
                C.broadcast_(out, h.root, engine=True)
                h.result = out
        elif kind == ALLTOALL:
            for h in hs:
                if tl: tl.activity(h.name, "ALLTOALL")
                h.result = C.alltoall(h.tensor, h.splits, engine=True)
        else:
            raise ValueError(f"unknown collective kind {kind}")

    # ----------------------------------------------------------- completion
    def synchronize(self, h: Handle):
        h.done.wait()
        if h.error is not None:
            raise h.error
        if h.done_event is not None:
            torch.cuda.current_stream().wait_event(h.done_event)
        return h.result

    def poll(self, h: Handle) -> bool:
        if not h.done.is_set():
            return False
        if h.done_event is not None:
            return h.done_event.query()
        return True


def _coll_phase(t: torch.Tensor) -> str:
    return "NCCL_ALLREDUCE" if t.is_cuda else "GLOO_ALLREDUCE"
