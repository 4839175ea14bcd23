"""Native CPU data plane: ``mivod._mvcore.Ring`` (csrc/engine/ring.cc).

Horovod 0.18.1 moves CPU tensors with MPI (``ops/mpi_operations.cc``) and sums
float16 with its own ``half.cc`` MPI op.  mivod has no
MPI: each process opens one listening socket, publishes ``host:port`` in the
torch.distributed rendezvous store, connects to its ring successor and accepts
its predecessor.  Allreduce is ring reduce-scatter + allgather (2(N-1)/N of the
buffer per rank on the wire), broadcast a pipelined chain, allgather the ring
all-gather with per-rank block sizes.  fp16 sums go through F16C, bf16 through
fp32 with round-to-nearest-even — natively, without gloo's fp32 round trip.

Two independent rings exist per process: one for the caller's thread (static
gradient schedule, broadcasts, metric averaging) and one for the engine's
background thread (named async ops), so the two never interleave on a socket.
``MIVOD_CPU_TRANSPORT=gloo`` switches CPU tensors back to torch's gloo groups.
"""
from __future__ import annotations

import os
import socket
from typing import List, Optional

import torch

_CODE = {torch.float32: 0, torch.float64: 1, torch.float16: 2, torch.bfloat16: 3,
         torch.int32: 4, torch.int64: 5, torch.uint8: 6, torch.int8: 7, torch.bool: 6}


def supported(t: torch.Tensor) -> bool:
    return (not t.is_cuda) and t.dtype in _CODE


def _local_addr() -> str:
    """Address the other ranks can reach this one at: MIVOD_RING_HOST, else the
    interface that routes to MASTER_ADDR (loopback stays loopback)."""
    h = os.environ.get("MIVOD_RING_HOST")
    if h:
        return h
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if master in ("127.0.0.1", "localhost", "::1"):
        return "127.0.0.1"
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect((master, int(os.environ.get("MASTER_PORT", "29500"))))
        addr = s.getsockname()[0]
        s.close()
        return addr
    except OSError:
        return socket.gethostbyname(socket.gethostname())


class TcpRing:
    def __init__(self, rank: int, size: int, store, tag: str, timeout_s: float = 300.0):
        from .. import _mvcore  # type: ignore
        self.rank, self.size = rank, size
        self.ring = _mvcore.Ring(rank, size, timeout_s)
        port = self.ring.listen()
        store.set(f"mivod/ring/{tag}/{rank}", f"{_local_addr()}:{port}")
        nxt = (rank + 1) % size
        host, p = store.get(f"mivod/ring/{tag}/{nxt}").decode().rsplit(":", 1)
        self.ring.connect(host, int(p))
        io_timeout = float(os.environ.get("HOROVOD_STALL_SHUTDOWN_TIME_SECONDS", "0") or 0)
        if io_timeout > 0:
            self.ring.set_timeout(io_timeout)

    # ---------------------------------------------------------------- ops
    def allreduce_(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In-place sum (``average``: / size for floating dtypes)."""
        work = t if t.is_contiguous() else t.contiguous()
        if work.dtype == torch.bool:
            w = work.to(torch.uint8)
            self.ring.allreduce(w.data_ptr(), w.numel(), _CODE[torch.uint8], False)
            work.copy_(w != 0)
        else:
            fp = work.dtype.is_floating_point
            self.ring.allreduce(work.data_ptr(), work.numel(), _CODE[work.dtype], average and fp)
            if average and not fp:
                work.floor_divide_(self.size)
        if work is not t:
            t.copy_(work)
        return t

    def broadcast_(self, t: torch.Tensor, root: int) -> torch.Tensor:
        work = t if t.is_contiguous() else t.contiguous()
        self.ring.broadcast(work.data_ptr(), work.numel() * work.element_size(), int(root))
        if work is not t:
            t.copy_(work)
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate along dim 0; first dims may differ between ranks."""
        src = (t if t.dim() > 0 else t.reshape(1)).contiguous()
        rows = torch.zeros(self.size, dtype=torch.int64)
        rows[self.rank] = src.shape[0]
        self.allreduce_(rows)
        rest = tuple(src.shape[1:])
        row_bytes = src.element_size() * (int(torch.tensor(rest).prod()) if rest else 1)
        out = torch.empty((int(rows.sum()),) + rest, dtype=src.dtype)
        self.ring.allgatherv(src.data_ptr(), out.data_ptr(),
                             [int(r) * row_bytes for r in rows.tolist()])
        return out

    def barrier(self):
        self.ring.barrier()

    def close(self):
        self.ring.close()


def make_rings(state, generation: int = 0) -> Optional[List[TcpRing]]:
    """(main ring, engine ring) for a multi-rank world, or None (gloo)."""
    if state.size <= 1 or os.environ.get("MIVOD_CPU_TRANSPORT", "ring").lower() == "gloo":
        return None
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store()
    t = float(os.environ.get("MIVOD_INIT_TIMEOUT_S", "300"))
    return [TcpRing(state.rank, state.size, store, f"{generation}/{tag}", t)
            for tag in ("main", "engine")]
