"""``import mivod.tensorflow.keras as hvd`` (== ``mivod.keras``)."""
from ...keras import *  # noqa: F401,F403
from ...keras import (DistributedOptimizer, broadcast_global_variables, broadcast_variables,
                      callbacks, load_model)  # noqa: F401
