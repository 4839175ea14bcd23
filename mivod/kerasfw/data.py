"""A small ``tf.data.Dataset`` work-alike for the TF2 reference script's input
pipeline (/root/reference/tensorflow2_keras_mnist.py:37-41):
``from_tensor_slices((x, y)).repeat().shuffle(10000).batch(128)``.

Elements are index-addressed, so shuffling permutes indices (tf.data's
buffer-shuffle semantics, exactly: a ``buffer_size`` reservoir over the
repeated stream) and batching gathers whole arrays at once."""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np


class Dataset:
    def __init__(self, arrays, index_stream_fn, batch=None, drop_remainder=False, fn=None,
                 length=None):
        self._arrays = arrays
        self._idx = index_stream_fn
        self._batch = batch
        self._drop = drop_remainder
        self._fn = fn
        self._len = length

    @staticmethod
    def from_tensor_slices(tensors):
        arrays = tuple(np.asarray(t) for t in (tensors if isinstance(tensors, (tuple, list))
                                               else (tensors,)))
        n = len(arrays[0])
        if any(len(a) != n for a in arrays):
            raise ValueError("all tensors must have the same first dimension")
        return Dataset(arrays, lambda: iter(range(n)), length=n)

    def repeat(self, count: Optional[int] = None):
        base = self._idx

        def gen():
            k = 0
            while count is None or k < count:
                yield from base()
                k += 1
        n = None if count is None or self._len is None else self._len * count
        return Dataset(self._arrays, gen, self._batch, self._drop, self._fn, n)

    def shuffle(self, buffer_size: int, seed: Optional[int] = None,
                reshuffle_each_iteration: bool = True):
        base = self._idx
        rng_seed = [seed]

        def gen():
            rng = np.random.default_rng(rng_seed[0])
            buf = []
            for i in base():
                if len(buf) < buffer_size:
                    buf.append(i)
                    continue
                j = int(rng.integers(buffer_size))
                yield buf[j]
                buf[j] = i
            rng.shuffle(buf)
            yield from buf
        return Dataset(self._arrays, gen, self._batch, self._drop, self._fn, self._len)

    def batch(self, batch_size: int, drop_remainder: bool = False):
        n = None
        if self._len is not None:
            n = self._len // batch_size if drop_remainder else -(-self._len // batch_size)
        return Dataset(self._arrays, self._idx, batch_size, drop_remainder, self._fn, n)

    def map(self, fn: Callable):
        prev = self._fn
        f = fn if prev is None else (lambda *a: fn(*prev(*a)))
        return Dataset(self._arrays, self._idx, self._batch, self._drop, f, self._len)

    def take(self, count: int):
        base = self._idx
        per = self._batch or 1

        def gen():
            for k, i in enumerate(base()):
                if k >= count * per:
                    return
                yield i
        return Dataset(self._arrays, gen, self._batch, self._drop, self._fn,
                       count if self._len is None else min(count, self._len))

    def prefetch(self, buffer_size=None):
        return self

    def __len__(self):
        if self._len is None:
            raise TypeError("dataset length is unknown (infinite)")
        return self._len

    def _emit(self, idx):
        sel = np.asarray(idx)
        out = tuple(a[sel] for a in self._arrays)
        if self._fn is not None:
            out = self._fn(*out)
            if not isinstance(out, tuple):
                out = (out,)
        return out if len(out) > 1 else out[0]

    def __iter__(self):
        if self._batch is None:
            for i in self._idx():
                yield self._emit(i)
            return
        buf = []
        for i in self._idx():
            buf.append(i)
            if len(buf) == self._batch:
                yield self._emit(buf)
                buf = []
        if buf and not self._drop:
            yield self._emit(buf)

    def shard(self, num_shards: int, index: int):
        base = self._idx

        def gen():
            for k, i in enumerate(base()):
                if k % num_shards == index:
                    yield i
        n = None if self._len is None else len(range(index, self._len, num_shards))
        return Dataset(self._arrays, gen, self._batch, self._drop, self._fn, n)
