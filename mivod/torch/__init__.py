"""``import mivod.torch as hvd`` — horovod.torch-compatible API on PyTorch-ROCm.

Parity: horovod 0.18.1 ``horovod/torch``.
"""
from ..common.basics import (comm_stream, cross_rank, cross_size, device, gloo_enabled, init, is_initialized,
                             local_rank, local_size, mpi_enabled, mpi_threads_supported,
                             nccl_built, rank, rocm_built, shutdown, size)
from ..ops.compression import Compression
from .functions import (allgather_object, broadcast_object, broadcast_optimizer_state,
                        broadcast_parameters)
from .mpi_ops import (Adasum, Average, HorovodInternalError, Sum, allgather, allgather_async,
                      allreduce, allreduce_, allreduce_async, allreduce_async_, alltoall,
                      alltoall_async, broadcast, broadcast_, broadcast_async, broadcast_async_,
                      join, poll, synchronize)
from .optimizer import DistributedOptimizer
from .graphs import GraphedStep, make_graphed_step
