"""Keras callbacks: the ones the reference attaches on rank 0 —
``ModelCheckpoint('checkpoint-{epoch}.h5')`` and ``TensorBoard(log_dir,
update_freq='batch')`` (/root/reference/mnist_keras.py:100-105,
/root/reference/tensorflow2_keras_mnist.py:85-89) — plus ``History``,
``LearningRateScheduler``, ``ReduceLROnPlateau``, ``EarlyStopping``,
``CSVLogger``, ``LambdaCallback`` and the progress logger.
"""
from __future__ import annotations

import csv
import json
import os
import sys
import time
from typing import Dict, List, Optional

import numpy as np

from . import backend as K


class Callback:
    def __init__(self):
        self.model = None
        self.params: Dict = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_batch_begin(self, batch, logs=None): pass
    def on_batch_end(self, batch, logs=None): pass
    def on_train_batch_begin(self, batch, logs=None): self.on_batch_begin(batch, logs)
    def on_train_batch_end(self, batch, logs=None): self.on_batch_end(batch, logs)
    def on_test_begin(self, logs=None): pass
    def on_test_end(self, logs=None): pass


class CallbackList:
    def __init__(self, callbacks: List[Callback], model, params):
        self.callbacks = list(callbacks)
        for c in self.callbacks:
            c.set_model(model)
            c.set_params(params)

    def __getattr__(self, hook):
        def call(*a, **kw):
            for c in self.callbacks:
                getattr(c, hook)(*a, **kw)
        return call


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history: Dict[str, list] = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class ProgbarLogger(Callback):
    """Per-epoch summary line (keras ``verbose=1/2`` style) on stdout."""

    def __init__(self, verbose=1):
        super().__init__()
        self.verbose = verbose

    def on_epoch_begin(self, epoch, logs=None):
        self.t0 = time.time()
        if self.verbose:
            print(f"Epoch {epoch + 1}/{self.params.get('epochs')}", flush=True)

    def on_epoch_end(self, epoch, logs=None):
        if self.verbose:
            dt = time.time() - self.t0
            steps = self.params.get("steps") or 0
            items = " - ".join(f"{k}: {v:.4f}" for k, v in (logs or {}).items()
                               if isinstance(v, (float, int, np.floating)))
            print(f"{steps}/{steps} - {dt:.0f}s - {items}", flush=True)


def _fmt_path(filepath, epoch, logs):
    return filepath.format(epoch=epoch + 1, **{k: v for k, v in (logs or {}).items()
                                               if isinstance(v, (int, float, np.floating))})


class ModelCheckpoint(Callback):
    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False,
                 save_weights_only=False, mode="auto", period=1, save_freq="epoch"):
        super().__init__()
        self.filepath = filepath
        self.monitor = monitor
        self.verbose = verbose
        self.save_best_only = save_best_only
        self.save_weights_only = save_weights_only
        self.period = period
        self.mode = mode
        self.best = None
        self._since = 0

    def _better(self, cur):
        if self.best is None:
            return True
        maxish = self.mode == "max" or (self.mode == "auto" and "acc" in self.monitor)
        return cur > self.best if maxish else cur < self.best

    def on_epoch_end(self, epoch, logs=None):
        self._since += 1
        if self._since < self.period:
            return
        self._since = 0
        path = _fmt_path(self.filepath, epoch, logs)
        if self.save_best_only:
            cur = (logs or {}).get(self.monitor)
            if cur is None or not self._better(cur):
                return
            self.best = cur
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save(path)
        if self.verbose:
            print(f"\nEpoch {epoch + 1}: saving model to {path}")


class TensorBoard(Callback):
    """Scalar logging to TensorBoard event files (+ a JSONL mirror)."""

    def __init__(self, log_dir="./logs", update_freq="epoch", **kw):
        super().__init__()
        self.log_dir = log_dir
        self.update_freq = update_freq
        self._step = 0
        self.writer = None
        self.jsonl = None

    def on_train_begin(self, logs=None):
        from .tfevents import EventWriter
        os.makedirs(self.log_dir, exist_ok=True)
        self.writer = EventWriter(os.path.join(self.log_dir, "train"))
        self.jsonl = open(os.path.join(self.log_dir, "scalars.jsonl"), "a")

    def _write(self, step, logs, prefix):
        sc = {f"{prefix}{k}": float(v) for k, v in (logs or {}).items()
              if isinstance(v, (int, float, np.floating)) and k not in ("batch", "size")}
        if not sc:
            return
        self.writer.add_scalars(step, sc)
        self.jsonl.write(json.dumps({"step": step, **sc}) + "\n")

    def on_batch_end(self, batch, logs=None):
        self._step += 1
        freq = self.update_freq
        if freq == "batch" or (isinstance(freq, int) and self._step % freq == 0):
            self._write(self._step, logs, "batch_")

    def on_epoch_end(self, epoch, logs=None):
        self._write(epoch, logs, "epoch_")
        self.writer.flush()
        self.jsonl.flush()

    def on_train_end(self, logs=None):
        if self.writer:
            self.writer.close()
        if self.jsonl:
            self.jsonl.close()


class LearningRateScheduler(Callback):
    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule = schedule
        self.verbose = verbose

    def on_epoch_begin(self, epoch, logs=None):
        lr = K.get_value(self.model.optimizer.lr)
        try:
            new = self.schedule(epoch, lr)
        except TypeError:
            new = self.schedule(epoch)
        K.set_value(self.model.optimizer.lr, new)
        if self.verbose:
            print(f"\nEpoch {epoch + 1}: LearningRateScheduler setting learning rate to {new}.")

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs["lr"] = K.get_value(self.model.optimizer.lr)


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="val_loss", factor=0.1, patience=10, verbose=0, mode="auto",
                 min_delta=1e-4, cooldown=0, min_lr=0.0):
        super().__init__()
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.min_delta, self.cooldown, self.min_lr, self.verbose = min_delta, cooldown, min_lr, verbose
        self.maxish = mode == "max" or (mode == "auto" and "acc" in monitor)
        self.best, self.wait, self.cool = None, 0, 0

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        better = self.best is None or (cur > self.best + self.min_delta if self.maxish
                                       else cur < self.best - self.min_delta)
        if self.cool > 0:
            self.cool -= 1
            self.wait = 0
        if better:
            self.best, self.wait = cur, 0
        elif self.cool == 0:
            self.wait += 1
            if self.wait >= self.patience:
                old = K.get_value(self.model.optimizer.lr)
                new = max(old * self.factor, self.min_lr)
                K.set_value(self.model.optimizer.lr, new)
                if self.verbose:
                    print(f"\nEpoch {epoch + 1}: ReduceLROnPlateau reducing learning rate to {new}.")
                self.cool, self.wait = self.cooldown, 0


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", min_delta=0, patience=0, mode="auto", **kw):
        super().__init__()
        self.monitor, self.min_delta, self.patience = monitor, abs(min_delta), patience
        self.maxish = mode == "max" or (mode == "auto" and "acc" in monitor)
        self.best, self.wait = None, 0

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        better = self.best is None or (cur > self.best + self.min_delta if self.maxish
                                       else cur < self.best - self.min_delta)
        if better:
            self.best, self.wait = cur, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                self.model.stop_training = True


class CSVLogger(Callback):
    def __init__(self, filename, separator=",", append=False):
        super().__init__()
        self.filename, self.sep, self.append = filename, separator, append
        self.writer = None

    def on_epoch_end(self, epoch, logs=None):
        logs = {k: v for k, v in (logs or {}).items()}
        if self.writer is None:
            self.f = open(self.filename, "a" if self.append else "w", newline="")
            self.keys = sorted(logs)
            self.writer = csv.DictWriter(self.f, ["epoch"] + self.keys, delimiter=self.sep)
            if not self.append:
                self.writer.writeheader()
        self.writer.writerow({"epoch": epoch, **{k: logs.get(k) for k in self.keys}})
        self.f.flush()

    def on_train_end(self, logs=None):
        if self.writer is not None:
            self.f.close()


class LambdaCallback(Callback):
    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None,
                 on_batch_end=None, on_train_begin=None, on_train_end=None):
        super().__init__()
        for n, f in dict(on_epoch_begin=on_epoch_begin, on_epoch_end=on_epoch_end,
                         on_batch_begin=on_batch_begin, on_batch_end=on_batch_end,
                         on_train_begin=on_train_begin, on_train_end=on_train_end).items():
            if f is not None:
                setattr(self, n, f)
