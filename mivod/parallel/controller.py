"""Controller factory: the C++ TCP coordinator (``mivod._mvcore.Controller``)."""
from __future__ import annotations


def make_controller(state, cfg):
    from .native_controller import NativeController
    return NativeController(state, cfg)
