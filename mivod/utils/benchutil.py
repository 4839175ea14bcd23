"""Self-diagnosis for the benchmark scripts (bench.py, benchmarks/bench_bert.py).

A multi-GPU run that hangs or silently runs on fewer ranks than asked should
say so: this module

* defaults the RCCL watchdog (``MIVOD_RCCL_TIMEOUT_S``) and horovod's
  ``HOROVOD_STALL_SHUTDOWN_TIME_SECONDS`` for multi-rank benchmark runs, so a
  stuck collective makes every rank exit non-zero with the collective's name
  instead of burning the driver's time limit (the library defaults stay
  horovod-compatible: no timeout);
* reports what RCCL itself sees (run-time / header version, ``ncclCommCount``,
  CTA range) next to ``hvd.size()``;
* turns the per-bucket timing events the DistributedOptimizer records around
  every collective (``time_comm``) into measured allreduce time per step and
  algorithm / bus bandwidth (busbw = algbw * 2(N-1)/N, the ring convention).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

MULTI_RANK_TIMEOUT_S = "300"


def world_size_from_env(environ=None) -> int:
    env = os.environ if environ is None else environ
    for k in ("HOROVOD_SIZE", "WORLD_SIZE", "OMPI_COMM_WORLD_SIZE"):
        v = env.get(k)
        if v not in (None, ""):
            return int(v)
    return 1


def multi_rank_defaults(environ=None) -> Dict[str, str]:
    """Before ``hvd.init()``: for a multi-rank run, default the RCCL watchdog
    timeout and the stall-shutdown time (user settings win).  Returns what was set."""
    env = os.environ if environ is None else environ
    if world_size_from_env(env) <= 1:
        return {}
    applied = {}
    for k in ("MIVOD_RCCL_TIMEOUT_S", "HOROVOD_STALL_SHUTDOWN_TIME_SECONDS"):
        if env.get(k, "") == "":
            env[k] = MULTI_RANK_TIMEOUT_S
            applied[k] = MULTI_RANK_TIMEOUT_S
    return applied


def rccl_info() -> Optional[dict]:
    """What the GPU data plane of this process is (None without one)."""
    from ..common import basics
    st = basics.state()
    tr = st.gpu
    out: dict = {"transport": st.backend, "hvd_size": st.size}
    try:
        from .. import _mvcomm  # type: ignore
        out["version"] = int(_mvcomm.rccl_version())
        out["header_version"] = int(_mvcomm.header_version())
        note = _mvcomm.version_note()
        if note:
            out["version_note"] = note
    except Exception:
        pass
    if tr is None:
        out["nranks"] = None
        return out
    if hasattr(tr, "count"):
        out["nranks"] = tr.count()                     # ncclCommCount
        out["ctas"] = list(tr.ctas)
        out["timeout_s"] = basics.rccl_timeout_s()
    else:
        out["nranks"] = tr.size
    if st.mesh is not None:
        out["mesh"] = {"max_bytes": st.mesh.capacity, "timeout_s": st.mesh.mesh.timeout_s,
                       "oneshot_max_bytes": st.mesh.mesh.oneshot_max_bytes}
    return out


def comm_timing_record(timings: Sequence[tuple], steps: int, size: int) -> dict:
    """``timings``: [(bucket, payload bytes, ms)] over ``steps`` timed steps ->
    measured allreduce time per step, per-bucket mean time, algbw / busbw (GB/s)."""
    if not timings or steps <= 0:
        return {"allreduce_ms": None, "algbw_GBps": None, "busbw_GBps": None, "per_bucket": []}
    per: Dict[str, List] = {}
    order: List[str] = []
    tot_ms = tot_b = 0.0
    for name, nb, ms in timings:
        if name not in per:
            per[name] = [int(nb), 0.0, 0]
            order.append(name)
        per[name][1] += float(ms)
        per[name][2] += 1
        tot_ms += float(ms)
        tot_b += float(nb)
    fac = 2.0 * (size - 1) / size if size > 1 else 1.0
    rows = []
    for name in order:
        nb, ms, k = per[name]
        mean = ms / k
        alg = nb / (mean * 1e-3) / 1e9 if mean > 0 else None
        rows.append({"bucket": name, "bytes": nb, "ms": round(mean, 4),
                     "busbw_GBps": round(alg * fac, 2) if alg else None})
    alg = tot_b / (tot_ms * 1e-3) / 1e9 if tot_ms > 0 else None
    return {"allreduce_ms": round(tot_ms / steps, 4),
            "algbw_GBps": round(alg, 2) if alg else None,
            "busbw_GBps": round(alg * fac, 2) if alg else None,
            "per_bucket": rows}
