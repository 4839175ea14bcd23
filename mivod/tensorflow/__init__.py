"""``mivod.tensorflow`` namespace: ``mivod.tensorflow.keras`` mirrors
``horovod.tensorflow.keras`` (the TF2 reference script's import,
/root/reference/tensorflow2_keras_mnist.py:18) on mivod's Keras front end."""
