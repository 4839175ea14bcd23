"""Process-level state: ``init``/``shutdown``/``rank``/``size``/``local_rank`` ...

Parity: horovod 0.18.1 ``horovod/common/basics.py``, as used
by /root/reference/mnist_keras.py:30,35,42,84 and
/root/reference/tensorflow2_keras_mnist.py:25,32,35,55.

MI355X design: one process per GPU.  ``init()`` pins the process to GPU
``local_rank`` (the reference does this by hand with TF session config,
mnist_keras.py:32-36), rendezvouses through torch's TCP store (a gloo world
that also serves CPU tensors), creates mivod's OWN RCCL communicator eagerly
(``transport.RcclTransport`` — unique id published by rank 0 in the store,
``ncclCommInitRank`` in C++, riding xGMI inside a node; horovod's lazy
NCCL-comm creation), intra-/cross-node child comms by
``ncclCommSplit`` for hierarchical allreduce, the native TCP rings for CPU
tensors, and a high-priority HIP stream on which every GPU collective — the
gradient buckets and the engine's named ops alike, in one cross-rank-agreed
order (``parallel.order``) — and every fused optimizer step runs, overlapped
with backward on the compute stream.  At size 1 no network is touched
(``MIVOD_FORCE_COLLECTIVES=1`` still builds a 1-rank RCCL comm so the GPU
collective path can be exercised on one GPU).

``MIVOD_TRANSPORT``: ``rccl`` (default with a GPU) | ``torch`` (torch's
ProcessGroupNCCL, A/B only) | ``gloo-gpu`` (GPU compute, gloo wire — several
ranks on ONE GPU, the multi-rank GPU test mode) | ``gloo`` / ``cpu`` (no GPU).
"""
from __future__ import annotations

import atexit
import datetime
import logging
import os
import threading

import torch
import torch.distributed as dist

from .config import Config

log = logging.getLogger("mivod")

_NOT_INIT = "Horovod has not been initialized; use hvd.init()."


class _State:
    def __init__(self):
        self.initialized = False
        self.rank = 0
        self.size = 1
        self.local_rank = 0
        self.local_size = 1
        self.cross_rank = 0
        self.cross_size = 1
        self.config: Config | None = None
        self.device = torch.device("cpu")
        self.backend = "none"
        self.pg = None           # torch.distributed world (rendezvous, CPU fallback)
        self.cpu_pg = None       # gloo group for CPU tensors
        self.engine_cpu_pg = None  # gloo group for the named-op engine's CPU tensors
        self.local_pg = None     # intra-node gloo group (hierarchical CPU ops)
        self.cross_pg = None     # one rank per node with equal local_rank
        self.gpu = None          # GPU transport (RcclTransport / PgTransport)
        self.gpu_local = None    # ncclCommSplit intra-node child
        self.gpu_cross = None    # ncclCommSplit cross-node child
        self.mesh = None         # xGMI mesh one-shot allreduce (small buckets)
        self.comm_stream = None
        self.rings = None        # native CPU data plane: [main ring, engine ring] (tcp_ring.py)
        self.init_count = 0
        self.owns_pg = False
        self.engine = None
        self.store_kind = "none"  # rendezvous: "native" (launcher's KV store) | "torch"
        self.lock = threading.RLock()


_state = _State()


def _first_env(names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return v
    return default


def resolve_topology(env=None) -> dict:
    """Rank / size / local / cross topology from the environment.

    Understands mivodrun / horovodrun (``HOROVOD_*``), torchrun (``RANK``,
    ``LOCAL_RANK`` ...) and Open MPI (``OMPI_COMM_WORLD_*``) launchers.
    """
    old = None
    if env is not None:
        old = dict(os.environ)
        os.environ.clear()
        os.environ.update(env)
    try:
        rank = int(_first_env(["HOROVOD_RANK", "RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK"], 0))
        size = int(_first_env(["HOROVOD_SIZE", "WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE"], 1))
        local_rank = int(_first_env(["HOROVOD_LOCAL_RANK", "LOCAL_RANK",
                                     "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID"], 0))
        local_size = int(_first_env(["HOROVOD_LOCAL_SIZE", "LOCAL_WORLD_SIZE",
                                     "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"], size))
        cross_size = int(_first_env(["HOROVOD_CROSS_SIZE", "GROUP_WORLD_SIZE"],
                                    max(1, size // max(1, local_size))))
        cross_rank = int(_first_env(["HOROVOD_CROSS_RANK", "GROUP_RANK"],
                                    rank // max(1, local_size)))
    finally:
        if old is not None:
            os.environ.clear()
            os.environ.update(old)
    if not (0 <= rank < size):
        raise ValueError(f"invalid rank {rank} for size {size}")
    if not (0 <= local_rank < local_size):
        raise ValueError(f"invalid local_rank {local_rank} for local_size {local_size}")
    return dict(rank=rank, size=size, local_rank=local_rank, local_size=local_size,
                cross_rank=cross_rank, cross_size=cross_size)


def _gpu_available() -> bool:
    if os.environ.get("MIVOD_TRANSPORT", "").lower() in ("gloo", "tcp", "cpu", "local"):
        return False
    try:
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover
        return False


def init(comm=None, process_sets=None):
    """Initialize mivod.  Idempotent.  ``comm`` is accepted for API parity
    (horovod accepted an mpi4py communicator); a list of ranks is not supported."""
    del process_sets
    with _state.lock:
        if _state.initialized:
            return
        if comm is not None and not isinstance(comm, (list, tuple)) and comm is not True:
            log.debug("mivod.init: ignoring MPI communicator argument (no MPI in mivod)")
        cfg = Config.from_env()
        _state.config = cfg
        from ..utils import logging as mvlog
        mvlog.configure(cfg)

        if dist.is_available() and dist.is_initialized():
            # Adopt an existing torch.distributed world (e.g. started by the user).
            topo = resolve_topology()
            topo["rank"] = dist.get_rank()
            topo["size"] = dist.get_world_size()
            _state.owns_pg = False
        else:
            topo = resolve_topology()
            _state.owns_pg = True
        _state.rank = topo["rank"]
        _state.size = topo["size"]
        _state.local_rank = topo["local_rank"]
        _state.local_size = topo["local_size"]
        _state.cross_rank = topo["cross_rank"]
        _state.cross_size = topo["cross_size"]

        use_gpu = _gpu_available()
        if use_gpu:
            ndev = torch.cuda.device_count()
            dev_index = _state.local_rank % ndev
            torch.cuda.set_device(dev_index)
            _state.device = torch.device("cuda", dev_index)
            prio = -1 if cfg.comm_priority == "high" else 0
            _state.comm_stream = torch.cuda.Stream(device=_state.device, priority=prio)
        else:
            _state.device = torch.device("cpu")

        transport = cfg.transport or ("rccl" if use_gpu else "gloo")
        if transport == "nccl":
            transport = "rccl"
        from ..parallel.order import ORDER
        _state.gpu = _state.gpu_local = _state.gpu_cross = _state.mesh = None
        _state.init_count += 1
        if _state.size > 1:
            if not dist.is_initialized():
                backend = "nccl" if (use_gpu and transport == "torch") else "gloo"
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
                tmo = float(os.environ.get("MIVOD_INIT_TIMEOUT_S", "600"))
                kwargs = dict(backend=backend, rank=_state.rank, world_size=_state.size,
                              timeout=datetime.timedelta(seconds=tmo))
                # launched by mivodrun: bootstrap through the launcher's native
                # rendezvous store (csrc/engine/store.cc) instead of torch's TCPStore
                from ..run.store import from_env as _native_store
                store = _native_store(tmo)
                if store is not None:
                    kwargs["store"] = store
                    _state.store_kind = "native"
                else:
                    _state.store_kind = "torch"
                if backend == "nccl":
                    kwargs["device_id"] = _state.device
                dist.init_process_group(**kwargs)
            world_backend = dist.get_backend()
            _state.pg = dist.group.WORLD
            _state.cpu_pg = _state.pg if world_backend == "gloo" else dist.new_group(backend="gloo")
            # the engine's CPU named ops get their own gloo group / TCP ring so they
            # never interleave on a socket with the caller thread's CPU collectives
            _state.engine_cpu_pg = dist.new_group(backend="gloo")
            _make_hierarchy_groups()
            from ..parallel.tcp_ring import make_rings
            _state.rings = make_rings(_state, generation=_state.init_count)
            if use_gpu:
                _make_gpu_plane(transport, world_backend, cfg)
                _make_mesh()
            else:
                _state.backend = "gloo"
        else:
            _state.backend = "local"
            if use_gpu and os.environ.get("MIVOD_FORCE_COLLECTIVES", "0") == "1":
                from ..parallel.transport import RcclTransport
                _state.gpu = RcclTransport.create(
                    0, 1, _state.device,
                    timeout_s=rccl_timeout_s(cfg))
                _state.backend = "rccl"
        ORDER.reset(enabled=_state.gpu is not None and _state.size > 1)
        _state.initialized = True

        from ..parallel.engine import Engine
        _state.engine = Engine(_state)
        _state.engine.start()
        atexit.register(shutdown)


def _hierarchical_topology() -> bool:
    ls, cs = _state.local_size, _state.cross_size
    return ls * cs == _state.size and ls != _state.size and ls != 1


def _make_gpu_plane(transport: str, world_backend: str, cfg) -> None:
    """The GPU transport of a multi-rank world (+ hierarchical children)."""
    from ..parallel.transport import PgTransport, RcclTransport
    if transport == "rccl":
        store = dist.distributed_c10d._get_default_store()
        timeout = rccl_timeout_s(cfg)
        ctas = int(os.environ.get("MIVOD_RCCL_CTAS", "0") or 0)

        def make(c: int, tag: str = "") -> "RcclTransport":
            return RcclTransport.create(
                _state.rank, _state.size, _state.device, store,
                key=f"mivod/rccl/{_state.init_count}{tag}", timeout_s=timeout,
                exit_on_abort=cfg.stall_shutdown_time_s > 0, min_ctas=c, max_ctas=c)

        if cfg.autotune and ctas == 0 and _state.size > 1:
            # channel count autotune: one communicator per candidate, keep the fastest
            from ..parallel.autotune import tune_rccl_ctas
            mb = 2 ** 20
            sizes = [cfg.first_bucket_mb * mb, cfg.bucket_mb * mb, cfg.last_bucket_mb * mb]
            _state.gpu, best, res = tune_rccl_ctas(
                lambda c: make(c, f"/cta{c}"), lambda t: t.time_allreduce(sizes),
                log_path=cfg.autotune_log)
            log.info("RCCL CTA autotune: %s -> %s", res, best or "default")
        else:
            _state.gpu = make(ctas)
        _state.backend = "rccl"
        if _hierarchical_topology():
            _state.gpu_local = _state.gpu.split(_state.cross_rank, _state.local_rank)
            _state.gpu_cross = _state.gpu.split(_state.local_rank, _state.cross_rank)
        return
    if transport == "torch":
        pg = _state.pg if world_backend == "nccl" else dist.new_group(backend="nccl")
        _state.gpu = PgTransport(pg, staged=False, name="torch-nccl")
        _state.backend = "torch-nccl"
        sub_backend, staged = "nccl", False
    elif transport in ("gloo-gpu", "gloo_gpu"):
        _state.gpu = PgTransport(dist.new_group(backend="gloo"), staged=True, name="gloo-gpu")
        _state.backend = "gloo-gpu"
        sub_backend, staged = "gloo", True
    else:
        raise ValueError(f"unknown MIVOD_TRANSPORT={transport!r} "
                         "(rccl | torch | gloo-gpu | gloo)")
    if _hierarchical_topology():
        ls, cs = _state.local_size, _state.cross_size
        for node in range(cs):
            ranks = list(range(node * ls, (node + 1) * ls))
            g = dist.new_group(ranks=ranks, backend=sub_backend)
            if _state.rank in ranks:
                _state.gpu_local = PgTransport(g, staged=staged, name=_state.gpu.name)
        for lr in range(ls):
            ranks = [node * ls + lr for node in range(cs)]
            g = dist.new_group(ranks=ranks, backend=sub_backend)
            if _state.rank in ranks:
                _state.gpu_cross = PgTransport(g, staged=staged, name=_state.gpu.name)


def rccl_timeout_s(cfg=None) -> float:
    """The RCCL watchdog timeout: ``MIVOD_RCCL_TIMEOUT_S``, else horovod's
    ``HOROVOD_STALL_SHUTDOWN_TIME_SECONDS`` (0 = no timeout, horovod's default;
    bench.py sets both for multi-rank runs)."""
    cfg = cfg or _state.config or Config.from_env()
    v = os.environ.get("MIVOD_RCCL_TIMEOUT_S", "")
    return float(v) if v not in ("", None) else float(cfg.stall_shutdown_time_s or 0.0)


def _make_mesh() -> None:
    """MIVOD_MESH_MAX_MB > 0 and every rank on this node: the xGMI mesh allreduce
    serves buckets up to that size (csrc/comm/mesh.hip) — one-shot up to
    MIVOD_MESH_ONESHOT_KB (default 1024), two-shot above."""
    mb = float(os.environ.get("MIVOD_MESH_MAX_MB", "0") or 0)
    if mb <= 0 or _state.local_size != _state.size or _state.size > 16:
        return
    from ..parallel.transport import MeshTransport
    store = dist.distributed_c10d._get_default_store()
    tmo = float(os.environ.get("MIVOD_MESH_TIMEOUT_S", "") or rccl_timeout_s() or 30.0)
    one_kb = float(os.environ.get("MIVOD_MESH_ONESHOT_KB", "1024") or 1024)
    _state.mesh = MeshTransport(_state.rank, _state.size, _state.device, int(mb * 2 ** 20), store,
                                key=f"mivod/mesh/{_state.init_count}", timeout_s=tmo,
                                exit_on_timeout=os.environ.get("MIVOD_MESH_TIMEOUT_EXIT", "1")
                                != "0", oneshot_max_bytes=int(one_kb * 1024))


def _make_hierarchy_groups():
    """Intra-node and cross-node gloo groups (hierarchical CPU allreduce).
    Every rank must create every group, in the same order."""
    ls, cs = _state.local_size, _state.cross_size
    if not _hierarchical_topology():
        return
    backend = "gloo"
    for node in range(cs):
        ranks = list(range(node * ls, (node + 1) * ls))
        g = dist.new_group(ranks=ranks, backend=backend)
        if _state.rank in ranks:
            _state.local_pg = g
    for lr in range(ls):
        ranks = [node * ls + lr for node in range(cs)]
        g = dist.new_group(ranks=ranks, backend=backend)
        if _state.rank in ranks:
            _state.cross_pg = g


def shutdown():
    with _state.lock:
        if not _state.initialized:
            return
        if _state.engine is not None:
            try:
                _state.engine.stop()
            except Exception as e:  # pragma: no cover
                log.warning("mivod engine shutdown error: %s", e)
            _state.engine = None
        if _state.comm_stream is not None:
            try:
                torch.cuda.current_stream().wait_stream(_state.comm_stream)
                torch.cuda.synchronize()
            except Exception:  # pragma: no cover
                pass
        if _state.rings:
            for r in _state.rings:
                r.close()
            _state.rings = None
        for tr in (_state.mesh, _state.gpu_local, _state.gpu_cross, _state.gpu):
            if tr is not None:
                try:
                    tr.close()
                except Exception as e:  # pragma: no cover
                    log.warning("mivod GPU transport shutdown error: %s", e)
        _state.gpu = _state.gpu_local = _state.gpu_cross = _state.mesh = None
        if _state.owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # pragma: no cover
                pass
        _state.initialized = False
        _state.pg = _state.cpu_pg = _state.engine_cpu_pg = None
        _state.local_pg = _state.cross_pg = None


def is_initialized() -> bool:
    return _state.initialized


def _check():
    if not _state.initialized:
        raise ValueError(_NOT_INIT)


def size() -> int:
    _check()
    return _state.size


def local_size() -> int:
    _check()
    return _state.local_size


def rank() -> int:
    _check()
    return _state.rank


def local_rank() -> int:
    _check()
    return _state.local_rank


def cross_rank() -> int:
    _check()
    return _state.cross_rank


def cross_size() -> int:
    _check()
    return _state.cross_size


def mpi_threads_supported() -> bool:
    """Parity stub: mivod has no MPI; its control plane is thread-safe."""
    _check()
    return True


def mpi_enabled() -> bool:
    return False


def gloo_enabled() -> bool:
    return True


def nccl_built() -> bool:
    """True when mivod's RCCL data plane (mivod._mvcomm) is importable."""
    try:
        from .. import _mvcomm  # noqa: F401
        return True
    except ImportError:
        return False


def rocm_built() -> bool:
    return torch.version.hip is not None


def device() -> torch.device:
    _check()
    return _state.device


def comm_stream():
    _check()
    return _state.comm_stream


def state() -> _State:
    return _state
