"""``import horovod.torch as hvd`` → :mod:`mivod.torch` (horovod 0.18.1 ``horovod/torch`` API)."""
from mivod.torch import *  # noqa: F401,F403
from mivod.torch import (Adasum, Average, Compression, DistributedOptimizer,  # noqa: F401
                         HorovodInternalError, Sum, allgather, allgather_async, allgather_object,
                         allreduce, allreduce_, allreduce_async, allreduce_async_, alltoall,
                         alltoall_async, broadcast, broadcast_, broadcast_async, broadcast_async_,
                         broadcast_object, broadcast_optimizer_state, broadcast_parameters,
                         cross_rank, cross_size, init, is_initialized, join, local_rank,
                         local_size, mpi_threads_supported, poll, rank, shutdown, size,
                         synchronize)
