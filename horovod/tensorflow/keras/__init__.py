"""``import horovod.tensorflow.keras as hvd`` → :mod:`mivod.tensorflow.keras`
(/root/reference/tensorflow2_keras_mnist.py:18,25,58,71-82)."""
from mivod.tensorflow.keras import *  # noqa: F401,F403
from mivod.tensorflow.keras import (DistributedOptimizer,  # noqa: F401
                                    broadcast_global_variables, broadcast_variables, load_model)

from . import callbacks  # noqa: F401,E402
