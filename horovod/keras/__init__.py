"""``import horovod.keras as hvd`` → :mod:`mivod.keras` (horovod 0.18.1 ``horovod/keras`` API,
as used by /root/reference/mnist_keras.py:20,30,87,97)."""
from mivod.keras import *  # noqa: F401,F403
from mivod.keras import (DistributedOptimizer, broadcast_global_variables,  # noqa: F401
                         broadcast_variables, load_model)

from . import callbacks  # noqa: F401,E402
