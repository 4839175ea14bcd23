"""horovod Keras callbacks.

* ``BroadcastGlobalVariablesCallback(root_rank)`` — after the FIRST batch
  (so lazily-created optimizer slots exist) overwrite every rank's model
  variables and optimizer state with ``root_rank``'s
  (/root/reference/mnist_keras.py:93-98, tensorflow2_keras_mnist.py:67-71).
* ``MetricAverageCallback()`` — at epoch end, allreduce-average every entry of
  ``logs`` in sorted key order, in place, before later callbacks see them
  (tensorflow2_keras_mnist.py:73-77).
* ``LearningRateScheduleCallback`` / ``LearningRateWarmupCallback`` — Goyal et
  al. gradual warmup (arXiv 1706.02677) applied per batch with optional
  momentum correction (tensorflow2_keras_mnist.py:79-82).
"""
from __future__ import annotations

import warnings

import torch

from ..common import basics
from ..kerasfw import backend as K
from ..kerasfw.callbacks import Callback
from ..torch import mpi_ops as _ops


class BroadcastGlobalVariablesCallback(Callback):
    def __init__(self, root_rank: int = 0, device: str = ""):
        super().__init__()
        self.root_rank = root_rank
        self.device = device
        self.broadcast_done = False

    def on_batch_end(self, batch, logs=None):
        if self.broadcast_done:
            return
        from . import broadcast_global_variables
        broadcast_global_variables(self.root_rank, model=self.model)
        self.broadcast_done = True


class MetricAverageCallback(Callback):
    def __init__(self, device: str = ""):
        super().__init__()
        self.device = device

    def _average_metrics_in_place(self, logs):
        logs = logs if logs is not None else {}
        keys = [k for k in sorted(logs) if isinstance(logs[k], (int, float))
                or (hasattr(logs[k], "item") and getattr(logs[k], "size", 1) == 1)]
        if not keys or basics.size() == 1:
            return
        vec = torch.tensor([float(logs[k]) for k in keys], dtype=torch.float64)
        avg = _ops.allreduce(vec, name="MetricAverageCallback", op=_ops.Average)
        for k, v in zip(keys, avg.tolist()):
            logs[k] = v

    def on_epoch_end(self, epoch, logs=None):
        self._average_metrics_in_place(logs)


class LearningRateScheduleCallback(Callback):
    def __init__(self, multiplier, start_epoch=0, end_epoch=None, staircase=True,
                 momentum_correction=True, steps_per_epoch=None, initial_lr=None):
        super().__init__()
        self.start_epoch = start_epoch
        self.end_epoch = end_epoch
        self.staircase = staircase
        self.momentum_correction = momentum_correction
        self.initial_lr = initial_lr
        self.restore_momentum = None
        self.steps_per_epoch = steps_per_epoch
        self.current_epoch = None
        if not callable(multiplier):
            self.staircase = True
            self.multiplier = lambda epoch: multiplier
        else:
            self.multiplier = multiplier

    def _autodetect_steps_per_epoch(self):
        if self.params.get("steps"):
            return self.params["steps"]
        if self.params.get("samples") and self.params.get("batch_size"):
            return self.params["samples"] // self.params["batch_size"]
        raise ValueError("Could not autodetect the number of steps per epoch. Please specify "
                         f"the steps_per_epoch parameter to the {type(self).__name__}().")

    def _adjust_learning_rate(self, epoch):
        old_lr = K.get_value(self.model.optimizer.lr)
        new_lr = self.initial_lr * self.multiplier(epoch)
        K.set_value(self.model.optimizer.lr, new_lr)
        if hasattr(self.model.optimizer, "momentum") and self.momentum_correction:
            # momentum correction (Goyal et al. §2.1): scale momentum by lr ratio for this step
            self.restore_momentum = K.get_value(self.model.optimizer.momentum)
            K.set_value(self.model.optimizer.momentum, self.restore_momentum * new_lr / old_lr)

    def _restore_momentum_if_needed(self):
        if self.restore_momentum:
            K.set_value(self.model.optimizer.momentum, self.restore_momentum)
            self.restore_momentum = None

    def on_train_begin(self, logs=None):
        if self.initial_lr is None:
            self.initial_lr = K.get_value(self.model.optimizer.lr)
        if not self.staircase and not self.steps_per_epoch:
            self.steps_per_epoch = self._autodetect_steps_per_epoch()

    def on_epoch_begin(self, epoch, logs=None):
        self.current_epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self.current_epoch < self.start_epoch or (self.end_epoch is not None and
                                                     self.current_epoch >= self.end_epoch):
            return
        if self.staircase and batch == 0:
            self._adjust_learning_rate(self.current_epoch)
        elif not self.staircase:
            self._adjust_learning_rate(self.current_epoch + float(batch) / self.steps_per_epoch)

    def on_batch_end(self, batch, logs=None):
        self._restore_momentum_if_needed()

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs["lr"] = K.get_value(self.model.optimizer.lr)


class LearningRateWarmupCallback(LearningRateScheduleCallback):
    """lr ramps from ``lr/size`` to ``lr`` over ``warmup_epochs`` epochs:
    ``multiplier(e) = (1/size) * (e' * (size - 1) / warmup_epochs + 1)`` with
    ``e' = epoch + batch/steps_per_epoch + 1/steps_per_epoch``."""

    def __init__(self, warmup_epochs=5, momentum_correction=True, steps_per_epoch=None,
                 verbose=0, initial_lr=None):
        def multiplier(epoch):
            # shifted by one step so the lr curve ends exactly on epoch boundaries
            epoch += 1.0 / self.steps_per_epoch
            n = basics.size()
            return 1.0 / n * (epoch * (n - 1) / warmup_epochs + 1)

        super().__init__(multiplier, start_epoch=0, end_epoch=warmup_epochs, staircase=False,
                         momentum_correction=momentum_correction,
                         steps_per_epoch=steps_per_epoch, initial_lr=initial_lr)
        self.verbose = verbose

    def on_epoch_end(self, epoch, logs=None):
        super().on_epoch_end(epoch, logs)
        if epoch == self.end_epoch - 1 and self.verbose > 0:
            new_lr = K.get_value(self.model.optimizer.lr)
            print("\nEpoch %d: finished gradual learning rate warmup to %g." % (epoch + 1, new_lr))
