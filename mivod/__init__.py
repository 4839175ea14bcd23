"""mivod — an MI355X-native data-parallel training engine with the Horovod API.

``import mivod as hvd`` (or ``mivod.torch`` / ``mivod.keras``) gives
``init/rank/size/local_rank``, named async collectives with negotiation and
tensor fusion, ``DistributedOptimizer`` (hook path with a static bucket
schedule on RCCL/xGMI and hand-written gfx950 fused kernels), state broadcast,
Adasum, fp16/bf16 compression, a horovod-compatible timeline and stall
inspector, and the ``mivodrun`` / ``horovodrun`` launcher.  See SURVEY.md.
"""
__version__ = "0.1.0"

from .common.basics import (cross_rank, cross_size, device, gloo_enabled, init, is_initialized,
                            local_rank, local_size, mpi_enabled, mpi_threads_supported,
                            nccl_built, rank, rocm_built, shutdown, size)
from .ops.compression import Compression
from .torch import (Adasum, Average, DistributedOptimizer, HorovodInternalError, Sum, allgather,
                    allgather_async, allgather_object, allreduce, allreduce_, allreduce_async,
                    allreduce_async_, alltoall, alltoall_async, broadcast, broadcast_,
                    broadcast_async, broadcast_async_, broadcast_object,
                    broadcast_optimizer_state, broadcast_parameters, join, poll, synchronize)
