"""Horovod-compatible timeline (``HOROVOD_TIMELINE=/path/timeline.json``).

Parity: horovod ``common/timeline.cc``: a chrome://tracing
JSON where every tensor name is a "process" row and its phases (``NEGOTIATE_*``,
``QUEUE``, ``MEMCPY_IN_FUSION_BUFFER``, ``NCCL_ALLREDUCE``,
``MEMCPY_OUT_FUSION_BUFFER`` ...) are duration events; written by rank 0 only.
The writer is native (``mivod._mvcore.Timeline``: lock-free-ish queue + writer
thread); this module is the thin Python front.  ``HOROVOD_TIMELINE_MARK_CYCLES``
adds an instant event per engine cycle.  GPU phases additionally emit roctx
ranges (``mivod._mvk.range_push``) so ``rocprofv3 --marker-trace`` lines them up
with the mivod kernels and RCCL.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional

_TL = None
_LOCK = threading.Lock()


class _PyTimeline:
    """Fallback writer used only when the native core is unavailable."""

    def __init__(self, path: str, mark_cycles: bool):
        self.path = path
        self.mark_cycles = mark_cycles
        self.f = open(path, "w")
        self.f.write("[\n")
        self.lock = threading.Lock()
        self.t0 = time.perf_counter()
        self.pids = {}
        self.open = {}

    def _ts(self):
        return int((time.perf_counter() - self.t0) * 1e6)

    def _pid(self, name):
        pid = self.pids.get(name)
        if pid is None:
            pid = self.pids[name] = len(self.pids) + 1
            self._w({"name": "process_name", "ph": "M", "pid": pid, "args": {"name": name}})
            self._w({"name": "process_sort_index", "ph": "M", "pid": pid,
                     "args": {"sort_index": pid}})
        return pid

    def _w(self, ev):
        self.f.write(json.dumps(ev) + ",\n")

    def start(self, name, phase, args=None):
        with self.lock:
            pid = self._pid(name)
            if name in self.open:
                self._w({"ph": "E", "pid": pid, "tid": 1, "ts": self._ts()})
            ev = {"name": phase, "ph": "B", "pid": pid, "tid": 1, "ts": self._ts()}
            if args:
                ev["args"] = args
            self._w(ev)
            self.open[name] = phase

    def activity(self, name, phase):
        self.start(name, phase)

    def end(self, name):
        with self.lock:
            if name in self.open:
                self._w({"ph": "E", "pid": self._pid(name), "tid": 1, "ts": self._ts()})
                del self.open[name]

    def instant(self, name, what):
        with self.lock:
            self._w({"name": what, "ph": "i", "pid": self._pid(name), "tid": 1, "ts": self._ts(),
                     "s": "p"})

    def complete(self, name, phase, ts_us, dur_us):
        with self.lock:
            self._w({"name": phase, "ph": "X", "pid": self._pid(name), "tid": 2, "ts": int(ts_us),
                     "dur": max(0, int(dur_us))})

    def now_us(self):
        return self._ts()

    def mark_cycle(self):
        if self.mark_cycles:
            self.instant("cycle", "CYCLE_START")

    def close(self):
        with self.lock:
            if self.f:
                self.f.write("{}]\n")
                self.f.close()
                self.f = None


def start_timeline(path: str, mark_cycles: bool = False):
    """Start writing a timeline (rank 0 only, as horovod)."""
    global _TL
    from ..common import basics
    with _LOCK:
        if _TL is not None:
            return _TL
        if basics.is_initialized() and basics.rank() != 0:
            return None
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        try:
            from .. import _mvcore  # type: ignore
            _TL = _mvcore.Timeline(path, bool(mark_cycles))
        except Exception:
            _TL = _PyTimeline(path, mark_cycles)
        return _TL


def stop_timeline():
    global _TL, _REC
    with _LOCK:
        if _REC is not None:
            _REC.stop()
            _REC = None
        if _TL is not None:
            _TL.close()
            _TL = None


def get() -> Optional[object]:
    """The active timeline, starting it from ``HOROVOD_TIMELINE`` on first use."""
    global _TL
    if _TL is None:
        path = os.environ.get("HOROVOD_TIMELINE", "")
        if path:
            start_timeline(path, os.environ.get("HOROVOD_TIMELINE_MARK_CYCLES", "0")
                           not in ("", "0", "false"))
    return _TL


def note_plan(buckets):
    tl = get()
    if tl is None:
        return
    for b in buckets:
        tl.instant(b.name, f"PLAN {b.nbytes} bytes, {len(b.params)} tensors")


# ---------------------------------------------------------------------------
# GPU phases of the static gradient schedule
# ---------------------------------------------------------------------------
_REC = None


class PhaseRecorder:
    """Turns (start, end) timing-event pairs recorded on the compute / comm
    streams into timeline "X" events with GPU timestamps: per bucket
    ``MEMCPY_IN_FUSION_BUFFER`` (pack), ``NCCL_ALLREDUCE`` / ``ADASUM`` (the
    collective), ``OPTIMIZER_STEP`` (fused update) or ``MEMCPY_OUT_FUSION_BUFFER``.
    A daemon thread polls the end events, so the hot path never waits; on CPU
    tensors the phases are timed on the host."""

    def __init__(self, tl):
        self.tl = tl
        self.items = []
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self.ref = None          # (cuda event, timeline us at that event)
        self.running = True
        self.thread = threading.Thread(target=self._run, name="mivod-timeline-gpu", daemon=True)
        self.thread.start()

    def _ref(self):
        import torch
        if self.ref is None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            ev.synchronize()
            self.ref = (ev, self.tl.now_us())
        return self.ref

    def event(self):
        """A timing event recorded now on the current stream (None on CPU)."""
        import torch
        if not torch.cuda.is_available():
            return None
        self._ref()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def host(self):
        return self.tl.now_us()

    def add(self, name: str, phase: str, start, end):
        if start is None or end is None:
            return
        if isinstance(start, (int, float)):
            self.tl.complete(name, phase, int(start), int(end - start))
            return
        with self.cv:
            self.items.append((name, phase, start, end))
            self.cv.notify()

    def _run(self):
        while True:
            with self.cv:
                while self.running and not self.items:
                    self.cv.wait(0.05)
                if not self.running and not self.items:
                    return
                items, self.items = self.items, []
            keep = []
            for it in items:
                name, phase, s, e = it
                try:
                    if not e.query():
                        keep.append(it)
                        continue
                    ref_ev, ref_us = self.ref
                    ts = ref_us + ref_ev.elapsed_time(s) * 1000.0
                    dur = s.elapsed_time(e) * 1000.0
                    self.tl.complete(name, phase, int(ts), int(dur))
                except Exception:
                    pass
            if keep:
                with self.cv:
                    self.items = keep + self.items
                time.sleep(0.002)

    def stop(self):
        with self.cv:
            self.running = False
            self.cv.notify()
        self.thread.join(timeout=10)


def recorder() -> Optional[PhaseRecorder]:
    """The GPU phase recorder when a timeline is active on this rank (else None)."""
    global _REC
    tl = get()
    if tl is None:
        return None
    if _REC is None:
        with _LOCK:
            if _REC is None:
                _REC = PhaseRecorder(tl)
    return _REC
