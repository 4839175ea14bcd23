"""torch.distributed Store backed by mivod's native rendezvous KV store.

``mivod._mvcore.KVServer`` (csrc/engine/store.cc) runs in the launcher process
(``mivod.run.launcher.launch``), which exports its address as
``HOROVOD_GLOO_RENDEZVOUS_ADDR`` / ``HOROVOD_GLOO_RENDEZVOUS_PORT`` — the names
horovodrun uses for its Gloo rendezvous server.  Every rank's
``mivod.init()`` then bootstraps through ``NativeStore``: the gloo world
(``init_process_group(store=...)``), mivod's RCCL unique id, the xGMI mesh's IPC
handles and the TCP rings' addresses all go through the native store, not torch's
TCPStore.  Programs started by torchrun keep torch's env:// store (the agent owns
MASTER_PORT).
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch.distributed as dist


def _core():
    from .. import _mvcore  # type: ignore
    return _mvcore


def _b(v) -> bytes:
    if isinstance(v, bytes):
        return v
    if isinstance(v, str):
        return v.encode()
    return bytes(v)


class NativeStore(dist.Store):
    """A ``torch.distributed.Store`` over one ``KVClient`` connection."""

    def __init__(self, host: str, port: int, timeout_s: float = 300.0):
        super().__init__()
        self._c = _core().KVClient(host, int(port), float(timeout_s))
        self.host, self.port = host, int(port)

    # -- torch.distributed.Store interface (called by ProcessGroupGloo too) --
    def set(self, key, value):
        self._c.set(key, _b(value))

    def get(self, key):
        return self._c.get(key)

    def add(self, key, value):
        return int(self._c.add(key, int(value)))

    def compare_set(self, key, expected_value, desired_value):
        return self._c.compare_set(key, _b(expected_value), _b(desired_value))

    def check(self, keys: List[str]) -> bool:
        return bool(self._c.check(list(keys)))

    def wait(self, keys: List[str], timeout: Optional[datetime.timedelta] = None):
        t = timeout.total_seconds() if timeout is not None else self._c.timeout
        self._c.wait(list(keys), float(t))

    def delete_key(self, key) -> bool:
        return bool(self._c.delete_key(key))

    def num_keys(self) -> int:
        return int(self._c.num_keys())

    def set_timeout(self, timeout: datetime.timedelta):
        self._c.set_timeout(float(timeout.total_seconds()))

    def close(self):
        self._c.close()


def from_env(timeout_s: float = 300.0) -> Optional[NativeStore]:
    """The launcher's native store when ``HOROVOD_GLOO_RENDEZVOUS_ADDR/PORT`` are set
    (and ``MIVOD_STORE`` is not ``torch``), else None."""
    addr = os.environ.get("HOROVOD_GLOO_RENDEZVOUS_ADDR", "")
    port = os.environ.get("HOROVOD_GLOO_RENDEZVOUS_PORT", "")
    if not addr or not port or os.environ.get("MIVOD_STORE", "native") == "torch":
        return None
    return NativeStore(addr, int(port), timeout_s)


def serve(host: str = "0.0.0.0", port: int = 0):
    """Start a KVServer (the launcher's); returns it (``.port``, ``.close()``)."""
    return _core().KVServer(host, int(port))
