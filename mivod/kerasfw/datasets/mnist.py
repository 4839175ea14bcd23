"""``mnist.load_data()`` — real MNIST when a local ``mnist.npz`` exists,
otherwise a deterministic synthetic MNIST-shaped dataset (no network here).

The reference downloads MNIST (/root/reference/mnist_keras.py:48,
tensorflow2_keras_mnist.py:34-35, the latter to a per-rank path to avoid a
concurrent-download race).  This build host and the GPU boxes have no egress,
so when no file is found the data is *generated*: 28x28 uint8 seven-segment
renderings of the digits 0-9 with random translation (+-4 px), stroke width,
contrast and pixel noise — learnable like MNIST (a ConvNet reaches loss << 0.3
in one epoch) and identical on every rank (fixed seed), like the real file.
Real files are read with ``numpy.load(allow_pickle=False)``.
"""
from __future__ import annotations

import os

import numpy as np

#        a      b      c      d      e      f      g
_SEGS = {0: "abcdef", 1: "bc", 2: "abged", 3: "abgcd", 4: "fgbc", 5: "afgcd", 6: "afgedc",
         7: "abc", 8: "abcdefg", 9: "abcdfg"}


def _render(digit: int, thick: int) -> np.ndarray:
    img = np.zeros((28, 28), np.float32)
    top, mid, bot, left, right = 5, 13, 22, 9, 18
    t = thick
    seg = {
        "a": (slice(top, top + t), slice(left, right + 1)),
        "g": (slice(mid, mid + t), slice(left, right + 1)),
        "d": (slice(bot, bot + t), slice(left, right + 1)),
        "f": (slice(top, mid + t), slice(left, left + t)),
        "b": (slice(top, mid + t), slice(right - t + 1, right + 1)),
        "e": (slice(mid, bot + t), slice(left, left + t)),
        "c": (slice(mid, bot + t), slice(right - t + 1, right + 1)),
    }
    for s in _SEGS[digit]:
        img[seg[s]] = 1.0
    # soften edges (3x3 box blur)
    p = np.pad(img, 1)
    img = sum(p[i:i + 28, j:j + 28] for i in range(3) for j in range(3)) / 9.0
    return np.clip(img * 1.6, 0, 1)


def synthetic(n_train=60000, n_test=10000, seed=1234):
    rng = np.random.default_rng(seed)
    protos = np.stack([np.stack([_render(d, t) for d in range(10)]) for t in (2, 3)])

    def make(n):
        y = rng.integers(0, 10, n).astype(np.uint8)
        th = rng.integers(0, 2, n)
        x = protos[th, y]                               # [n, 28, 28]
        dx = rng.integers(-4, 5, n)
        dy = rng.integers(-3, 4, n)
        out = np.empty_like(x)
        for sx in range(-4, 5):
            for sy in range(-3, 4):
                m = (dx == sx) & (dy == sy)
                if m.any():
                    out[m] = np.roll(np.roll(x[m], sy, axis=1), sx, axis=2)
        contrast = rng.uniform(0.6, 1.0, (n, 1, 1)).astype(np.float32)
        noise = rng.normal(0, 0.08, out.shape).astype(np.float32)
        img = np.clip(out * contrast + noise, 0, 1)
        return (img * 255).astype(np.uint8), y

    x_train, y_train = make(n_train)
    x_test, y_test = make(n_test)
    return (x_train, y_train), (x_test, y_test)


def load_data(path: str = "mnist.npz"):
    candidates = [path, os.path.join(os.path.expanduser("~"), ".keras", "datasets", path),
                  os.environ.get("MIVOD_MNIST_NPZ", "")]
    for c in candidates:
        if c and os.path.isfile(c):
            with np.load(c, allow_pickle=False) as f:
                return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    return synthetic()
