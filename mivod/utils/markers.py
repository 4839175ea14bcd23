"""roctx ranges around mivod's gradient-path phases (``MIVOD_ROCTX=1``, or
implicitly when ``HOROVOD_TIMELINE`` is set).  View with
``rocprofv3 --marker-trace --kernel-trace``."""
from __future__ import annotations

import contextlib
import os

_ENABLED = None
_NAT = None


def enabled() -> bool:
    global _ENABLED, _NAT
    if _ENABLED is None:
        _ENABLED = os.environ.get("MIVOD_ROCTX", "0") not in ("", "0") or \
            bool(os.environ.get("HOROVOD_TIMELINE"))
        if _ENABLED:
            try:
                from .. import _mvk
                _NAT = _mvk
            except Exception:
                _ENABLED = False
    return _ENABLED


@contextlib.contextmanager
def range(name: str):
    if not enabled():
        yield
        return
    _NAT.range_push(name)
    try:
        yield
    finally:
        _NAT.range_pop()


def mark(name: str):
    if enabled():
        _NAT.mark(name)
