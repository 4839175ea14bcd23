"""``mivod.kerasfw`` — a Keras-compatible front end on PyTorch-ROCm.

TensorFlow / Keras are not installable in this environment (SURVEY.md §0,
§7.4 risk 2), yet the reference workloads are Keras scripts.  This package
keeps their API and behavioural contracts (``Sequential``, the layers the
reference uses, ``compile/fit/evaluate/save/load_model``, Keras optimizers
whose ``get_gradients`` is the horovod hook point, callbacks, ``datasets.mnist``,
``utils.to_categorical``, a ``tf.data``-like ``data.Dataset``) on PyTorch, so
``import mivod.kerasfw as keras`` + ``import mivod.keras as hvd`` runs the
reference scripts with only the imports changed (see examples/).
"""
from . import activations, backend, callbacks, data, datasets, layers, losses, optimizers, utils
from .models import Model, Sequential, load_model

__all__ = ["Sequential", "Model", "load_model", "layers", "optimizers", "losses", "callbacks",
           "datasets", "utils", "backend", "data", "activations"]
