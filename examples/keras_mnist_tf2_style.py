#!/usr/bin/env python3
"""Config 2 of BASELINE.json: the TF2 tf.keras MNIST trainer
(/root/reference/tensorflow2_keras_mnist.py) on mivod.

Recipe kept: per-rank data file name ``mnist-<rank>.npz``, a
``from_tensor_slices(...).repeat().shuffle(10000).batch(128)`` pipeline, Adam
lr 0.001*size, BroadcastGlobalVariablesCallback(0) + MetricAverageCallback() +
LearningRateWarmupCallback(warmup_epochs=3, verbose=1), rank-0 checkpoints and
TensorBoard, ``steps_per_epoch = 500 // size`` for 24 epochs.

    mivodrun -np 2 python examples/keras_mnist_tf2_style.py --epochs 4
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import mivod.kerasfw as keras  # noqa: E402
import mivod.tensorflow.keras as hvd  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=24)
    ap.add_argument("--steps", type=int, default=None, help="steps per epoch (default 500//size)")
    args = ap.parse_args(argv)

    base = os.environ.get("PS_MODEL_PATH", os.path.join(os.getcwd(), "models"))
    model_dir = os.path.abspath(os.path.join(base, "horovod-mnist"))

    hvd.init()
    (images, labels), _ = keras.datasets.mnist.load_data(path="mnist-%d.npz" % hvd.rank())
    ds = keras.data.Dataset.from_tensor_slices(
        ((images[..., np.newaxis] / 255.0).astype(np.float32), labels.astype(np.int64)))
    ds = ds.repeat().shuffle(10000).batch(128)

    model = keras.Sequential([
        keras.layers.Conv2D(32, [3, 3], activation="relu"),
        keras.layers.Conv2D(64, [3, 3], activation="relu"),
        keras.layers.MaxPooling2D(pool_size=(2, 2)),
        keras.layers.Dropout(0.25),
        keras.layers.Flatten(),
        keras.layers.Dense(128, activation="relu"),
        keras.layers.Dropout(0.5),
        keras.layers.Dense(10, activation="softmax"),
    ])
    opt = hvd.DistributedOptimizer(keras.optimizers.Adam(0.001 * hvd.size()))
    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(), optimizer=opt,
                  metrics=["accuracy"], experimental_run_tf_function=False)

    callbacks = [
        hvd.callbacks.BroadcastGlobalVariablesCallback(0),
        hvd.callbacks.MetricAverageCallback(),        # before any metric consumer
        hvd.callbacks.LearningRateWarmupCallback(warmup_epochs=3, verbose=1),
    ]
    if hvd.rank() == 0:
        callbacks.append(keras.callbacks.ModelCheckpoint(
            os.path.join(model_dir, "checkpoint-{epoch}.h5")))
        callbacks.append(keras.callbacks.TensorBoard(log_dir=model_dir, update_freq="batch"))
    steps = args.steps or 500 // hvd.size()
    hist = model.fit(ds, steps_per_epoch=steps, callbacks=callbacks, epochs=args.epochs,
                     verbose=1 if hvd.rank() == 0 else 0)
    return hist, model


if __name__ == "__main__":
    main()
    hvd.shutdown()
