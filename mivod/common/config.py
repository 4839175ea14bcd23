"""Environment knobs (Horovod-compatible names + mivod extensions).

Read once at ``mivod.init()``.  Horovod 0.18.1 semantics (SURVEY.md §5 "Config /
flag system"): ``HOROVOD_FUSION_THRESHOLD`` (bytes, default 64 MiB),
``HOROVOD_CYCLE_TIME`` (ms, default 5), ``HOROVOD_CACHE_CAPACITY`` (1024),
``HOROVOD_TIMELINE`` / ``HOROVOD_TIMELINE_MARK_CYCLES``, ``HOROVOD_AUTOTUNE`` /
``HOROVOD_AUTOTUNE_LOG``, ``HOROVOD_STALL_CHECK_TIME_SECONDS`` (60),
``HOROVOD_STALL_SHUTDOWN_TIME_SECONDS`` (0 = never), ``HOROVOD_STALL_CHECK_DISABLE``,
``HOROVOD_LOG_LEVEL``, ``HOROVOD_LOG_HIDE_TIME``, ``HOROVOD_HIERARCHICAL_ALLREDUCE``.

mivod extensions (MI355X-specific):
  ``MIVOD_BUCKET_MB``        gradient bucket size for the static DistributedOptimizer
                             schedule (default 32 MB; sized so an 8-rank ring over
                             one xGMI link finishes a bucket in well under 1 ms)
  ``MIVOD_FIRST_BUCKET_MB``  first (= last layers') bucket, small to start xGMI
                             traffic early (default 2 MB)
  ``MIVOD_LAST_BUCKET_MB``   last (= first layers') bucket, small so the exposed
                             allreduce + step after backward ends is short (4 MB)
  ``MIVOD_TRANSPORT``        ``rccl`` (default on GPU) | ``gloo`` (CPU)
  ``MIVOD_COMPRESSION``      default wire compression for DistributedOptimizer
  ``MIVOD_COMM_PRIORITY``    ``high`` (default) | ``normal`` HIP stream priority
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    return int(float(v))


def _env_float(name: str, default: float) -> float:
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    return float(v)


def _env_bool(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    return v.strip().lower() not in ("0", "false", "no", "off")


@dataclass
class Config:
    fusion_threshold: int = 64 * 1024 * 1024
    cycle_time_ms: float = 5.0
    cache_capacity: int = 1024
    timeline: str = ""
    timeline_mark_cycles: bool = False
    autotune: bool = False
    autotune_log: str = ""
    stall_check_disable: bool = False
    stall_check_time_s: float = 60.0
    stall_shutdown_time_s: float = 0.0
    log_level: str = "warning"
    log_hide_time: bool = False
    hierarchical_allreduce: bool = False
    bucket_mb: float = 32.0
    first_bucket_mb: float = 2.0
    last_bucket_mb: float = 4.0
    transport: str = ""
    compression: str = "none"
    comm_priority: str = "high"
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls) -> "Config":
        c = cls()
        c.fusion_threshold = _env_int("HOROVOD_FUSION_THRESHOLD", c.fusion_threshold)
        c.cycle_time_ms = _env_float("HOROVOD_CYCLE_TIME", c.cycle_time_ms)
        c.cache_capacity = _env_int("HOROVOD_CACHE_CAPACITY", c.cache_capacity)
        c.timeline = os.environ.get("HOROVOD_TIMELINE", "")
        c.timeline_mark_cycles = _env_bool("HOROVOD_TIMELINE_MARK_CYCLES")
        c.autotune = _env_bool("HOROVOD_AUTOTUNE")
        c.autotune_log = os.environ.get("HOROVOD_AUTOTUNE_LOG", "")
        c.stall_check_disable = _env_bool("HOROVOD_STALL_CHECK_DISABLE")
        c.stall_check_time_s = _env_float("HOROVOD_STALL_CHECK_TIME_SECONDS", c.stall_check_time_s)
        c.stall_shutdown_time_s = _env_float("HOROVOD_STALL_SHUTDOWN_TIME_SECONDS",
                                             c.stall_shutdown_time_s)
        c.log_level = os.environ.get("HOROVOD_LOG_LEVEL", c.log_level).lower()
        c.log_hide_time = _env_bool("HOROVOD_LOG_HIDE_TIME")
        c.hierarchical_allreduce = _env_bool("HOROVOD_HIERARCHICAL_ALLREDUCE")
        c.bucket_mb = _env_float("MIVOD_BUCKET_MB", c.bucket_mb)
        c.first_bucket_mb = _env_float("MIVOD_FIRST_BUCKET_MB", c.first_bucket_mb)
        c.last_bucket_mb = _env_float("MIVOD_LAST_BUCKET_MB", c.last_bucket_mb)
        c.transport = os.environ.get("MIVOD_TRANSPORT", "").lower()
        c.compression = os.environ.get("MIVOD_COMPRESSION", "none").lower()
        c.comm_priority = os.environ.get("MIVOD_COMM_PRIORITY", "high").lower()
        return c
