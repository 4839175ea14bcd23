"""``horovod.tensorflow`` namespace: only ``horovod.tensorflow.keras`` is provided (there is
no TensorFlow on PyTorch-ROCm; the Keras front end is :mod:`mivod.kerasfw`)."""
