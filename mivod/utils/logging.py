"""Rank-aware logging (parity: horovod ``common/logging.cc``, ``HOROVOD_LOG_LEVEL``
trace|debug|info|warning|error|fatal and ``HOROVOD_LOG_HIDE_TIME``)."""
from __future__ import annotations

import logging
import os
import sys

_LEVELS = {"trace": 5, "debug": logging.DEBUG, "info": logging.INFO,
           "warning": logging.WARNING, "warn": logging.WARNING, "error": logging.ERROR,
           "fatal": logging.CRITICAL}
_configured = False


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.mvrank = os.environ.get("HOROVOD_RANK", os.environ.get("RANK", "0"))
        return True


def configure(cfg=None):
    global _configured
    lg = logging.getLogger("mivod")
    level = _LEVELS.get((cfg.log_level if cfg else os.environ.get("HOROVOD_LOG_LEVEL", "warning")),
                        logging.WARNING)
    lg.setLevel(level)
    if _configured:
        return lg
    h = logging.StreamHandler(sys.stderr)
    hide = cfg.log_hide_time if cfg else False
    fmt = "[%(mvrank)s]<%(levelname)s> %(message)s" if hide else \
        "[%(asctime)s %(mvrank)s]<%(levelname)s> %(message)s"
    h.setFormatter(logging.Formatter(fmt))
    h.addFilter(_RankFilter())
    lg.addHandler(h)
    lg.propagate = False
    _configured = True
    return lg


def rank0_print(*args, **kwargs):
    """print() on rank 0 only (the reference gates verbosity on rank,
    /root/reference/mnist_keras.py:111)."""
    from ..common import basics
    if not basics.is_initialized() or basics.rank() == 0:
        print(*args, **kwargs)
