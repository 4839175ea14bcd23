"""``import horovod.tensorflow as hvd`` → :mod:`mivod.tensorflow` (the horovod.tensorflow API on
PyTorch-ROCm: allreduce with IndexedSlices, broadcast_global_variables, DistributedOptimizer,
DistributedGradientTape, BroadcastGlobalVariablesHook).  ``horovod.tensorflow.keras`` is the
Keras API on :mod:`mivod.kerasfw`."""
from mivod.tensorflow import *  # noqa: F401,F403
from mivod.tensorflow import __all__  # noqa: F401
