"""Process-level state: ``init``/``shutdown``/``rank``/``size``/``local_rank`` ...

Parity: horovod 0.18.1 ``horovod/common/basics.py``, as used
by /root/reference/mnist_keras.py:30,35,42,84 and
/root/reference/tensorflow2_keras_mnist.py:25,32,35,55.

MI355X design: one process per GPU.  ``init()`` pins the process to GPU
``local_rank`` (the reference does this by hand with TF session config,
mnist_keras.py:32-36), creates the RCCL communicator eagerly through
``torch.distributed`` (backend "nccl" == RCCL on ROCm, riding xGMI inside a
node), a gloo group for CPU tensors (metric averaging, tests), and a
high-priority HIP stream on which every gradient collective and fused optimizer
step runs, overlapped with backward on the compute stream.  At size 1 no
network is touched.
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
        self.pg = None           # main (GPU / default) group
        self.cpu_pg = None       # gloo group for CPU tensors
        self.engine_pg = None    # group used by the negotiated named-op engine
        self.engine_cpu_pg = None
        self.local_pg = None     # intra-node group (hierarchical ops)
        self.cross_pg = None     # one rank per node with equal local_rank
        self.comm_stream = None
        self.rings = None        # native CPU data plane: [main ring, engine ring] (tcp_ring.py)
        self.init_count = 0
        self.owns_pg = False
        self.engine = None
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
    if os.environ.get("MIVOD_TRANSPORT", "").lower() in ("gloo", "tcp", "cpu"):
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
        if _state.size > 1:
            if not dist.is_initialized():
                backend = "nccl" if (use_gpu and transport in ("rccl", "nccl")) else "gloo"
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
                kwargs = dict(backend=backend, rank=_state.rank, world_size=_state.size,
                              timeout=datetime.timedelta(
                                  seconds=float(os.environ.get("MIVOD_INIT_TIMEOUT_S", "600"))))
                if backend == "nccl":
                    kwargs["device_id"] = _state.device   # eager RCCL communicator init (C5/C6)
                dist.init_process_group(**kwargs)
            _state.backend = dist.get_backend()
            _state.pg = dist.group.WORLD
            if _state.backend == "gloo":
                _state.cpu_pg = _state.pg
            else:
                _state.cpu_pg = dist.new_group(backend="gloo")
            # Separate communicators for the negotiated engine so that its
            # background-thread collectives never interleave with the static
            # gradient schedule issued from backward hooks.
            _state.engine_pg = dist.new_group(backend=_state.backend) if _state.backend != "gloo" \
                else dist.new_group(backend="gloo")
            _state.engine_cpu_pg = dist.new_group(backend="gloo")
            _make_hierarchy_groups()
            from ..parallel.tcp_ring import make_rings
            _state.init_count += 1
            _state.rings = make_rings(_state, generation=_state.init_count)
        else:
            _state.backend = "local"
        _state.initialized = True

        from ..parallel.engine import Engine
        _state.engine = Engine(_state)
        _state.engine.start()
        atexit.register(shutdown)


def _make_hierarchy_groups():
    """Intra-node and cross-node groups (for hierarchical allreduce / Adasum).
    Every rank must create every group, in the same order."""
    ls, cs = _state.local_size, _state.cross_size
    if ls * cs != _state.size or ls == _state.size or ls == 1:
        return
    backend = _state.backend
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
        if _state.owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # pragma: no cover
                pass
        _state.initialized = False
        _state.pg = _state.cpu_pg = _state.engine_pg = _state.engine_cpu_pg = None
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
    """True when the RCCL (torch 'nccl') backend is available."""
    return dist.is_available() and dist.is_nccl_available()


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
