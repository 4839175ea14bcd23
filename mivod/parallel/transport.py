"""GPU data-plane transports.

``RcclTransport`` is the production path: mivod's own RCCL communicator
(``mivod._mvcomm``, csrc/comm/comm.cc) — created once per process from a unique
id that rank 0 publishes in the rendezvous store, driven from C++ on the
caller's HIP stream (the high-priority comm stream), watched by a C++ watchdog
thread (async errors + stalled collectives -> ncclCommAbort).  torch's
ProcessGroupNCCL is not involved.  Parity: horovod 0.18.1
``ops/nccl_operations.cc`` (the reference's GPU wire
is NCCL, /root/reference/README.md:57 ``-x NCCL_DEBUG=INFO``).

``PgTransport`` is the fallback over a torch.distributed group:
``MIVOD_TRANSPORT=torch`` (ProcessGroupNCCL, for A/B comparisons) and
``MIVOD_TRANSPORT=gloo-gpu`` (GPU compute, gloo wire staged through host memory
— the test mode that runs several ranks on ONE GPU, which RCCL refuses).

Both expose the same small interface on contiguous tensors; reduction ``op``
codes are the horovod ones from ``collectives`` (Average / Sum / Adasum are
resolved above this layer; here: SUM, AVG, MAX, MIN).
"""
from __future__ import annotations

from typing import List, Optional

import torch

SUM, AVG, MAX, MIN = "sum", "avg", "max", "min"


def _mvcomm():
    from .. import _mvcomm  # type: ignore
    return _mvcomm


def _dtype_code(dt: torch.dtype) -> int:
    m = _mvcomm()
    table = {torch.float32: m.FLOAT32, torch.float16: m.FLOAT16, torch.bfloat16: m.BFLOAT16,
             torch.float64: m.FLOAT64, torch.int32: m.INT32, torch.int64: m.INT64,
             torch.uint8: m.UINT8, torch.int8: m.INT8, torch.bool: m.UINT8}
    if dt not in table:
        raise TypeError(f"mivod RCCL transport: unsupported dtype {dt}")
    return table[dt]


def _op_code(op: str) -> int:
    m = _mvcomm()
    return {SUM: m.SUM, AVG: m.AVG, MAX: m.MAX, MIN: m.MIN}[op]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class RcclTransport:
    """mivod-owned RCCL communicator (one per process, plus ncclCommSplit children)."""

    name = "rccl"

    def __init__(self, comm):
        self.comm = comm
        self.rank = comm.rank
        self.size = comm.size

    @classmethod
    def create(cls, rank: int, size: int, device: torch.device, store=None, key: str = "",
               timeout_s: float = 0.0, exit_on_abort: bool = False, min_ctas: int = 0,
               max_ctas: int = 0) -> "RcclTransport":
        m = _mvcomm()
        if size == 1 or store is None:
            uid = m.unique_id()
        elif rank == 0:
            uid = m.unique_id()
            store.set(key, uid)
        else:
            uid = store.get(key)
        return cls(m.Comm(bytes(uid), rank, size, device.index, float(timeout_s),
                          bool(exit_on_abort), int(min_ctas), int(max_ctas)))

    def count(self) -> int:
        """ncclCommCount — the ranks RCCL itself sees (bench self-diagnosis)."""
        return int(self.comm.count())

    @property
    def ctas(self):
        """(minCTAs, maxCTAs) this communicator was created with (0: RCCL default)."""
        return self.comm.min_ctas, self.comm.max_ctas

    def time_allreduce(self, sizes_bytes, iters: int = 10, warmup: int = 3) -> float:
        """Seconds for one allreduce of each size in ``sizes_bytes`` (bf16 SUM, the
        bucket wire), MAX-reduced over ranks — the RCCL autotune objective."""
        dev = torch.device("cuda", self.comm.device)
        n = max(int(max(sizes_bytes)) // 2, 1)
        buf = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        views = [buf[:max(int(b) // 2, 1)] for b in sizes_bytes]
        for _ in range(warmup):
            for v in views:
                self.allreduce_(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            for v in views:
                self.allreduce_(v)
        e1.record()
        e1.synchronize()
        t = torch.tensor([e0.elapsed_time(e1) / 1e3 / iters], dtype=torch.float32, device=dev)
        self.allreduce_(t, MAX)
        return float(t.item())

    def split(self, color: int, key: int) -> Optional["RcclTransport"]:
        c = self.comm.split(color, key)
        return RcclTransport(c) if c is not None else None

    # ------------------------------------------------------------ collectives
    def allreduce_(self, t: torch.Tensor, op: str = SUM, prescale: float = 1.0) -> torch.Tensor:
        assert t.is_contiguous()
        n = t.numel()
        if n == 0:
            return t
        work = t.view(torch.uint8) if t.dtype == torch.bool else t
        dt = _dtype_code(work.dtype)
        p = work.data_ptr()
        if prescale != 1.0:
            if op not in (SUM, AVG):
                raise ValueError("prescale needs a sum/average reduction")
            if op == AVG:
                prescale = prescale / self.size
            self.comm.allreduce_premul(p, p, n, dt, float(prescale), _stream())
        elif op == AVG and not t.dtype.is_floating_point:
            self.comm.allreduce(p, p, n, dt, _op_code(SUM), _stream())
            t.floor_divide_(self.size)
        else:
            self.comm.allreduce(p, p, n, dt, _op_code(op), _stream())
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = SUM):
        self.comm.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(),
                                 _dtype_code(out.dtype), _op_code(op), _stream())

    def allgather_into(self, out: torch.Tensor, inp: torch.Tensor):
        """``out`` = concat of every rank's equally sized ``inp``."""
        self.comm.allgather(inp.data_ptr(), out.data_ptr(), inp.numel(), _dtype_code(inp.dtype),
                            _stream())

    def broadcast_(self, t: torch.Tensor, root: int) -> torch.Tensor:
        assert t.is_contiguous()
        work = t.view(torch.uint8) if t.dtype == torch.bool else t
        if work.numel():
            self.comm.broadcast(work.data_ptr(), work.data_ptr(), work.numel(),
                                _dtype_code(work.dtype), int(root), _stream())
        return t

    def sendrecv(self, send: torch.Tensor, recv: torch.Tensor, peer: int):
        self.comm.sendrecv(send.data_ptr(), send.numel(), recv.data_ptr(), recv.numel(),
                           _dtype_code(send.dtype), int(peer), _stream())

    def alltoallv(self, out: torch.Tensor, inp: torch.Tensor, send_counts: List[int],
                  recv_counts: List[int]):
        row = int(torch.tensor(inp.shape[1:]).prod()) if inp.dim() > 1 else 1
        sc = [c * row for c in send_counts]
        rc = [c * row for c in recv_counts]
        sd = [sum(sc[:i]) for i in range(len(sc))]
        rd = [sum(rc[:i]) for i in range(len(rc))]
        self.comm.alltoallv(inp.data_ptr(), sc, sd, out.data_ptr(), rc, rd,
                            _dtype_code(inp.dtype), _stream())

    def barrier(self, device: torch.device):
        x = torch.zeros(1, dtype=torch.int32, device=device)
        self.allreduce_(x, SUM)
        torch.cuda.current_stream().synchronize()

    # --------------------------------------------------------- observability
    def stats(self) -> dict:
        s = self.comm.stats()
        return {"calls": s.calls, "bytes": s.bytes, "completed": s.completed}

    def check(self):
        self.comm.check()

    def close(self):
        self.comm.destroy()


class PgTransport:
    """GPU tensors over a torch.distributed group (``torch`` = ProcessGroupNCCL,
    ``gloo-gpu`` = gloo staged through host memory)."""

    def __init__(self, pg, staged: bool, name: str):
        import torch.distributed as dist
        self.dist = dist
        self.pg = pg
        self.staged = staged
        self.name = name
        self.rank = dist.get_rank(pg)
        self.size = dist.get_world_size(pg)
        self._calls = 0
        self._bytes = 0

    def _rop(self, op):
        R = self.dist.ReduceOp
        return {SUM: R.SUM, AVG: R.AVG, MAX: R.MAX, MIN: R.MIN}[op]

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        h = t.detach().to("cpu")
        if h.dtype in (torch.bfloat16, torch.float16):
            h = h.float()
        if h.dtype == torch.bool:
            h = h.to(torch.uint8)
        return h

    def _count(self, t):
        self._calls += 1
        self._bytes += t.numel() * t.element_size()

    def allreduce_(self, t: torch.Tensor, op: str = SUM, prescale: float = 1.0) -> torch.Tensor:
        self._count(t)
        if prescale != 1.0:
            t.mul_(prescale)
        if not self.staged:
            if op == AVG and not t.dtype.is_floating_point:
                self.dist.all_reduce(t, op=self._rop(SUM), group=self.pg)
                t.floor_divide_(self.size)
            else:
                self.dist.all_reduce(t, op=self._rop(op), group=self.pg)
            return t
        h = self._host(t)
        self.dist.all_reduce(h, op=self._rop(SUM if op == AVG else op), group=self.pg)
        if op == AVG:
            if h.dtype.is_floating_point:
                h.div_(self.size)
            else:
                h.floor_divide_(self.size)
        t.copy_(h.to(t.device))
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = SUM):
        self._count(inp)
        if not self.staged:
            self.dist.reduce_scatter_tensor(out, inp, op=self._rop(op), group=self.pg)
            return
        h = self._host(inp)
        self.dist.all_reduce(h, op=self._rop(SUM if op == AVG else op), group=self.pg)
        if op == AVG:
            h.div_(self.size)
        n = out.numel()
        out.copy_(h[self.rank * n:(self.rank + 1) * n].to(out.device))

    def allgather_into(self, out: torch.Tensor, inp: torch.Tensor):
        self._count(inp)
        if not self.staged:
            self.dist.all_gather_into_tensor(out, inp, group=self.pg)
            return
        h = self._host(inp)
        parts = [torch.empty_like(h) for _ in range(self.size)]
        self.dist.all_gather(parts, h, group=self.pg)
        out.copy_(torch.cat(parts).to(out.device, out.dtype))

    def broadcast_(self, t: torch.Tensor, root: int) -> torch.Tensor:
        self._count(t)
        groot = self.dist.get_global_rank(self.pg, root) if self.pg is not None else root
        if not self.staged:
            self.dist.broadcast(t, src=groot, group=self.pg)
            return t
        h = self._host(t)
        self.dist.broadcast(h, src=groot, group=self.pg)
        t.copy_(h.to(t.device))
        return t

    def sendrecv(self, send: torch.Tensor, recv: torch.Tensor, peer: int):
        self._count(send)
        gpeer = self.dist.get_global_rank(self.pg, peer)
        s, r = send, recv
        if self.staged:
            s, r = send.detach().cpu(), torch.empty(recv.shape, dtype=recv.dtype)
            if s.dtype in (torch.bfloat16, torch.float16):   # gloo moves raw 16-bit words
                s, r = s.view(torch.int16), r.view(torch.int16)
        ops = []
        if s.numel():
            ops.append(self.dist.P2POp(self.dist.isend, s.contiguous(), gpeer, group=self.pg))
        if r.numel():
            ops.append(self.dist.P2POp(self.dist.irecv, r, gpeer, group=self.pg))
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()
        if self.staged and r.numel():
            recv.copy_(r.view(recv.dtype).to(recv.device))

    def alltoallv(self, out: torch.Tensor, inp: torch.Tensor, send_counts: List[int],
                  recv_counts: List[int]):
        self._count(inp)
        if not self.staged:
            self.dist.all_to_all_single(out, inp, recv_counts, send_counts, group=self.pg)
            return
        h = inp.detach().cpu()
        ho = torch.empty(out.shape, dtype=out.dtype)
        self.dist.all_to_all_single(ho, h, recv_counts, send_counts, group=self.pg)
        out.copy_(ho.to(out.device))

    def barrier(self, device: torch.device):
        self.dist.barrier(group=self.pg)
        torch.cuda.current_stream().synchronize()

    def stats(self) -> dict:
        return {"calls": self._calls, "bytes": self._bytes, "completed": self._calls}

    def check(self):
        pass

    def close(self):
        pass


class MeshTransport:
    """xGMI mesh allreduce (``mivod._mvcomm.Mesh``, csrc/comm/mesh.hip) for small
    and medium buckets: one-shot (every rank reads every peer's HIP-IPC-mapped
    staging copy and reduces locally) up to ``MIVOD_MESH_ONESHOT_KB``, two-shot
    (mesh reduce-scatter into IPC result buffers + all-gather from them) above,
    both in fixed rank order (bit-identical on all ranks).  Used for Sum/Average
    of fp32/bf16/fp16 buffers of at most ``MIVOD_MESH_MAX_MB``; all ranks must
    share one node.  A producer can write straight into the next call's staging
    slot (``stage_view``) — the bucket pack kernel does — saving the copy.

    A peer that does not arrive within ``timeout_s`` (``MIVOD_MESH_TIMEOUT_S``,
    default the RCCL watchdog timeout or 30 s) poisons the output with NaN, and
    the native watcher thread ends the process with a diagnosis — a rank never
    trains on its local gradient.  Parity: SURVEY.md §2.5 K7."""

    name = "mesh"
    _CODES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}

    def __init__(self, rank: int, size: int, device: torch.device, capacity_bytes: int, store,
                 key: str, timeout_s: float = 30.0, exit_on_timeout: bool = True,
                 oneshot_max_bytes: int = 2 ** 20):
        m = _mvcomm()
        self.rank, self.size = rank, size
        self.device = device
        self.mesh = m.Mesh(rank, size, device.index, int(capacity_bytes), float(timeout_s),
                           bool(exit_on_timeout))
        self.mesh.oneshot_max_bytes = int(oneshot_max_bytes)
        store.set(f"{key}/{rank}", self.mesh.handles())
        hs = [bytes(store.get(f"{key}/{r}")) for r in range(size)]
        self.mesh.open(hs)
        self.capacity = self.mesh.capacity

    def accepts(self, t: torch.Tensor, op: str) -> bool:
        return (op in (SUM, AVG) and t.dtype in self._CODES and t.is_contiguous()
                and t.numel() * t.element_size() <= self.capacity
                and t.data_ptr() % 16 == 0)

    def stage_view(self, numel: int, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """A tensor over the staging slot the NEXT allreduce reads (None if it
        does not fit): write the bucket there, then ``allreduce_into``."""
        if dtype not in self._CODES or numel * torch.empty((), dtype=dtype).element_size() \
                > self.capacity:
            return None
        from ..ops import kernels as K
        return K.tensor_from_ptr(self.mesh.stage_ptr(), numel, dtype, self.device)

    def allreduce_(self, t: torch.Tensor, op: str = SUM, prescale: float = 1.0) -> torch.Tensor:
        return self.allreduce_into(t, t, op, prescale)

    def allreduce_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = SUM,
                       prescale: float = 1.0, algo: int = 0) -> torch.Tensor:
        """out = reduce(inp) over the mesh; ``inp`` may be a ``stage_view``."""
        assert out.numel() == inp.numel() and out.dtype == inp.dtype
        scale = float(prescale) * (1.0 / self.size if op == AVG else 1.0)
        self.mesh.allreduce(inp.data_ptr(), out.data_ptr(), out.numel(), self._CODES[out.dtype],
                            scale, _stream(), algo)
        return out

    def status(self) -> int:
        return self.mesh.status()

    def stats(self) -> dict:
        return {"mesh_calls": self.mesh.calls, "mesh_bytes": self.mesh.bytes,
                "mesh_two_shot_calls": self.mesh.two_shot_calls,
                "mesh_copies_saved": self.mesh.copies_saved}

    def close(self):
        self.mesh.close()
