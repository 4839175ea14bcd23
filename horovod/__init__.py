"""``horovod`` import namespace backed by mivod (drop-in for horovod 0.18.1 users).

The reference imports ``horovod.keras`` (/root/reference/mnist_keras.py:20) and
``horovod.tensorflow.keras`` (/root/reference/tensorflow2_keras_mnist.py:18);
PyTorch users of horovod import ``horovod.torch``.  Each of those modules here
re-exports the corresponding mivod module, so existing scripts switch to the
MI355X engine without edits to their ``import ... as hvd`` line:

    import horovod.torch as hvd             # == mivod.torch
    import horovod.keras as hvd             # == mivod.keras  (Keras front end: mivod.kerasfw)
    import horovod.tensorflow.keras as hvd  # == mivod.tensorflow.keras

Every name resolves to the same object as in mivod (one runtime state, one
engine); nothing here re-implements anything.
"""
from mivod import __version__  # noqa: F401
from mivod.common.basics import (cross_rank, cross_size, gloo_enabled, init,  # noqa: F401
                                 is_initialized, local_rank, local_size, mpi_enabled,
                                 mpi_threads_supported, nccl_built, rank, rocm_built, shutdown,
                                 size)
