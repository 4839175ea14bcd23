"""Python side of the native coordinator (``mivod._mvcore.Controller``).

Rank 0 listens on an ephemeral port and publishes ``host:port`` in the
torch.distributed rendezvous store; the other ranks read it and connect, so the
control plane needs no extra launcher flags.  All network waits run with the
GIL released.
"""
from __future__ import annotations

import os

import torch.distributed as dist

from .. import _mvcore  # type: ignore


class NativeController:
    def __init__(self, state, cfg):
        c = _mvcore.ControllerConfig()
        c.rank = state.rank
        c.size = state.size
        c.fusion_threshold = int(cfg.fusion_threshold)
        c.stall_check = not cfg.stall_check_disable
        c.stall_check_s = float(cfg.stall_check_time_s)
        c.stall_shutdown_s = float(cfg.stall_shutdown_time_s)
        c.connect_timeout_s = float(os.environ.get("MIVOD_INIT_TIMEOUT_S", "300"))
        c.cache_capacity = max(0, int(cfg.cache_capacity))
        self.ctl = _mvcore.Controller(c)
        from ..utils import timeline as TL
        tl = TL.get()
        if tl is not None and isinstance(tl, _mvcore.Timeline):
            self.ctl.set_timeline(tl)
        if state.size == 1:
            return                      # 1-rank world: coordinate() locally, no sockets
        store = dist.distributed_c10d._get_default_store()
        key = "mivod/controller"
        if state.rank == 0:
            port = self.ctl.listen()
            host = os.environ.get("MIVOD_CONTROLLER_HOST", os.environ.get("MASTER_ADDR",
                                                                          "127.0.0.1"))
            store.set(key, f"{host}:{port}")
            self.ctl.connect(host, port)
        else:
            addr = store.get(key).decode()
            host, port = addr.rsplit(":", 1)
            self.ctl.connect(host, int(port))

    def negotiate(self, requests, shutdown=False, position=0):
        """-> (responses, all_shutdown, exec_at)"""
        return self.ctl.negotiate(list(requests), bool(shutdown), int(position))

    def last_stalls(self):
        return self.ctl.last_stalls()

    def close(self):
        self.ctl.close()
