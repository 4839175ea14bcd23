#!/usr/bin/env python3
"""Config 1 of BASELINE.json: the TF1/Keras MNIST ConvNet trainer
(/root/reference/mnist_keras.py) on mivod — Keras API on PyTorch-ROCm,
horovod API from ``mivod.keras``.

Same recipe: per-rank batch 128, Adadelta lr 1.0*size, epochs ceil(12/size),
ConvNet 32c3-64c3-maxpool-drop.25-fc128-drop.5-fc10 (1,199,882 params),
BroadcastGlobalVariablesCallback(0), rank-0 ModelCheckpoint + TensorBoard,
evaluation on every rank, rank-0 model save + serving export.

    python examples/keras_mnist_convnet.py                 # world 1
    mivodrun -np 2 python examples/keras_mnist_convnet.py --epochs 1
Extra flags (for CI): --epochs, --steps-per-epoch, --train-samples.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mivod.keras as hvd  # noqa: E402
import mivod.kerasfw as keras  # noqa: E402
from mivod.kerasfw import backend as K  # noqa: E402
from mivod.kerasfw.export import export_serving  # noqa: E402
from mivod.kerasfw.layers import Conv2D, Dense, Dropout, Flatten, MaxPooling2D  # noqa: E402


def build_convnet(input_shape, num_classes):
    net = keras.Sequential(name="mnist_convnet")
    net.add(Conv2D(32, kernel_size=(3, 3), activation="relu", input_shape=input_shape))
    net.add(Conv2D(64, (3, 3), activation="relu"))
    net.add(MaxPooling2D(pool_size=(2, 2)))
    net.add(Dropout(0.25))
    net.add(Flatten())
    net.add(Dense(128, activation="relu"))
    net.add(Dropout(0.5))
    net.add(Dense(num_classes, activation="softmax"))
    return net


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--train-samples", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--no-export", action="store_true")
    args = ap.parse_args(argv)

    base = os.environ.get("PS_MODEL_PATH", os.path.join(os.getcwd(), "models"))
    model_dir = os.path.abspath(os.path.join(base, "horovod-mnist"))
    export_dir = os.path.abspath(base)

    hvd.init()                                   # one process per GPU (pinned inside init)
    num_classes = 10
    epochs = args.epochs or int(math.ceil(12.0 / hvd.size()))

    (x_train, y_train), (x_test, y_test) = keras.datasets.mnist.load_data()
    rows, cols = 28, 28
    assert K.image_data_format() == "channels_last"
    x_train = x_train.reshape(-1, rows, cols, 1).astype("float32") / 255
    x_test = x_test.reshape(-1, rows, cols, 1).astype("float32") / 255
    if args.train_samples:
        x_train, y_train = x_train[:args.train_samples], y_train[:args.train_samples]
    if hvd.rank() == 0:
        print("x_train shape:", x_train.shape, f"({len(x_train)} train / {len(x_test)} test)")
    y_train = keras.utils.to_categorical(y_train, num_classes)
    y_test = keras.utils.to_categorical(y_test, num_classes)

    model = build_convnet((rows, cols, 1), num_classes)
    opt = hvd.DistributedOptimizer(keras.optimizers.Adadelta(1.0 * hvd.size()))
    model.compile(loss="categorical_crossentropy", optimizer=opt, metrics=["accuracy"])

    callbacks = [hvd.callbacks.BroadcastGlobalVariablesCallback(0)]
    if hvd.rank() == 0:     # rank 0 alone writes checkpoints and logs
        callbacks.append(keras.callbacks.ModelCheckpoint(
            os.path.join(model_dir, "checkpoint-{epoch}.h5")))
        callbacks.append(keras.callbacks.TensorBoard(log_dir=os.path.join(model_dir, "eval"),
                                                     update_freq="batch"))
    hist = model.fit(x_train, y_train, batch_size=args.batch_size, callbacks=callbacks,
                     epochs=epochs, verbose=1 if hvd.rank() == 0 else 0,
                     validation_data=(x_test, y_test))
    score = model.evaluate(x_test, y_test, verbose=0)

    if hvd.rank() == 0:
        saved = os.path.join(model_dir, "keras-sample-model.h5")
        model.save(saved)
        print("Model saved to {}".format(saved))
        if not args.no_export:
            reloaded = keras.load_model(saved)        # plain loader, as the reference
            print("Exported serving model to", export_serving(reloaded, export_dir))
    print("Test loss:", score[0])
    print("Test accuracy:", score[1])
    losses = hist.history.get("loss", [])
    if losses:
        print("mean train loss:", sum(losses) / len(losses))
    return hist, score


if __name__ == "__main__":
    main()
    hvd.shutdown()
