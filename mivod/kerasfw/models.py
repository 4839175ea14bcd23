"""Keras ``Sequential`` / ``Model`` on PyTorch: compile / fit / evaluate /
predict / save / load_model.

Training-loop contract kept from Keras (what the reference relies on,
/root/reference/mnist_keras.py:89-113, tensorflow2_keras_mnist.py:60-96):

* every step computes gradients through ``optimizer.get_gradients(loss,
  params)`` and applies them with ``optimizer.apply_gradients`` — the
  interception point horovod's Keras ``DistributedOptimizer`` overrides; there
  is no code path that bypasses it;
* callbacks see ``on_train_begin`` / ``on_epoch_begin`` / ``on_batch_begin`` /
  ``on_batch_end`` / ``on_epoch_end`` in list order with a mutable ``logs``
  dict (so ``MetricAverageCallback`` must come before checkpoint/TensorBoard);
* ``params`` carries ``steps`` / ``samples`` / ``batch_size`` for LR-schedule
  autodetection; numpy inputs are shuffled every epoch, the last partial batch
  is kept (60000 / 128 -> 469 steps per epoch).

Checkpoints are single safetensors files (weights, optimizer slots, JSON
architecture + optimizer config in the metadata) whatever the extension
(``checkpoint-{epoch}.h5`` keeps its name).
"""
from __future__ import annotations

import itertools
import json
import math
import time
import weakref
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import callbacks as cbks
from . import layers as L
from . import losses as LS
from . import optimizers as O


def _device():
    try:
        from ..common import basics
        if basics.is_initialized():
            return basics.device()
    except Exception:
        pass
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _to_tensor(a, dev, dtype=None):
    if torch.is_tensor(a):
        t = a
    else:
        t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None and t.is_floating_point():
        t = t.to(dtype)
    return t.to(dev, non_blocking=True)


# Live models in creation order: ``mivod.tensorflow.global_variables()`` (the
# tf.global_variables() collection horovod's broadcast_global_variables walks).
_LIVE_MODELS: "weakref.WeakSet" = weakref.WeakSet()
_model_seq = itertools.count()


class Model(nn.Module):
    """Keras-style model.  Subclass and implement ``call``, or use Sequential."""

    def __init__(self, name: Optional[str] = None):
        super().__init__()
        self._name = name or L._uid(type(self).__name__.lower())
        self.optimizer: Optional[O.Optimizer] = None
        self.loss = None
        self.metrics_names: List[str] = []
        self._metric_fns = []
        self.stop_training = False
        self.history = None
        self._compiled = False
        self._dev = None
        self._mvd_seq = next(_model_seq)
        _LIVE_MODELS.add(self)

    @property
    def name(self):
        return self._name

    # -- graph ---------------------------------------------------------------
    def call(self, x, training=False):
        raise NotImplementedError

    def _forward(self, x, training):
        """(output, logits-or-None) — logits when the last op is a softmax."""
        return self.call(x, training), None

    def forward(self, x, training: Optional[bool] = None):
        return self._forward(x, self.training if training is None else training)[0]

    def __call__(self, x, training: Optional[bool] = None):
        if not torch.is_tensor(x):
            x = _to_tensor(x, self.device_, torch.float32)
        return super().__call__(x, training)

    @property
    def device_(self):
        if self._dev is None:
            self._dev = _device()
        return self._dev

    @property
    def trainable_weights(self):
        return [p for p in self.parameters() if p.requires_grad]

    @property
    def variables(self):
        """All state (params + buffers), as horovod's eager broadcast path uses."""
        return [p for p in self.parameters()] + [b for b in self.buffers()
                                                 if b.is_floating_point()]

    def get_weights(self):
        out = []
        for m in self._keras_layers():
            out.extend(m.get_weights())
        return out

    def set_weights(self, weights):
        i = 0
        for m in self._keras_layers():
            n = len(m.get_weights())
            if n:
                m.set_weights(weights[i:i + n])
            i += n

    def _keras_layers(self):
        return [m for m in self.modules() if isinstance(m, L.Layer)]

    @property
    def layers(self):
        return self._keras_layers()

    def count_params(self):
        return sum(p.numel() for p in self.parameters())

    # -- compile ------------------------------------------------------------
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None,
                experimental_run_tf_function=None, run_eagerly=None, **kwargs):
        """``experimental_run_tf_function`` is accepted for parity with the TF2
        reference script (tensorflow2_keras_mnist.py:65); mivod's fit always
        goes through ``optimizer.get_gradients``."""
        self.optimizer = O.get(optimizer)
        self.loss = loss
        self._loss_fn = LS.get(loss)
        self._loss_kind = LS.kind(loss)
        self._metric_specs = list(metrics or [])
        self.metrics_names = ["loss"] + [m if isinstance(m, str) else getattr(m, "__name__", "m")
                                         for m in self._metric_specs]
        self._compiled = True
        self.to(self.device_)

    def _loss_value(self, y, out, logits):
        if logits is not None and self._loss_kind in ("categorical", "sparse") and \
                not getattr(self._loss_fn, "from_logits", False):
            if self._loss_kind == "categorical":
                return LS.categorical_crossentropy(y, logits, from_logits=True)
            return LS.sparse_categorical_crossentropy(y, logits, from_logits=True)
        return self._loss_fn(y, out)

    def _metric_values(self, y, out) -> Dict[str, torch.Tensor]:
        res = {}
        for spec, nm in zip(self._metric_specs, self.metrics_names[1:]):
            if spec in ("accuracy", "acc", "categorical_accuracy", "sparse_categorical_accuracy"):
                pred = out.argmax(-1)
                if self._loss_kind == "categorical" or spec == "categorical_accuracy":
                    tgt = y.argmax(-1)
                elif self._loss_kind == "binary":
                    pred = (out > 0.5).long().reshape(-1)
                    tgt = y.long().reshape(-1)
                else:
                    tgt = y.long().reshape(-1)
                res[nm] = (pred == tgt).float().mean()
            elif callable(spec):
                res[nm] = spec(y, out)
            else:
                raise ValueError(f"unknown metric {spec!r}")
        return res

    # -- steps ---------------------------------------------------------------
    def _train_step(self, xb, yb):
        out, logits = self._forward(xb, True)
        loss = self._loss_value(yb, out, logits)
        params = self.trainable_weights
        grads = self.optimizer.get_gradients(loss, params)
        self.optimizer.apply_gradients(zip(grads, params))
        with torch.no_grad():
            mets = self._metric_values(yb, out.detach())
        return loss.detach(), mets

    def _batches(self, x, y, batch_size, shuffle):
        n = len(x)
        idx = np.random.permutation(n) if shuffle else np.arange(n)
        idx_t = torch.from_numpy(idx).to(x.device)
        for b in range(int(math.ceil(n / batch_size))):
            sel = idx_t[b * batch_size:(b + 1) * batch_size]
            yield x.index_select(0, sel), y.index_select(0, sel)

    def _prep_xy(self, x, y):
        dev = self.device_
        xt = _to_tensor(x, dev, torch.float32)
        yt = _to_tensor(y, dev) if y is not None else None
        if yt is not None and yt.is_floating_point() and self._loss_kind in ("categorical",
                                                                             "regression"):
            yt = yt.float()
        return xt, yt

    @staticmethod
    def _is_dataset(x):
        return not isinstance(x, (np.ndarray, torch.Tensor, list)) and hasattr(x, "__iter__")

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None,
            validation_split=0.0, validation_data=None, shuffle=True, initial_epoch=0,
            steps_per_epoch=None, validation_steps=None, **kwargs):
        if not self._compiled:
            raise RuntimeError("You must compile your model before training/testing.")
        dataset = self._is_dataset(x)
        batch_size = batch_size or (None if dataset else 32)
        if dataset:
            it = iter(x)
            samples = None
            steps = steps_per_epoch
            if steps is None:
                try:
                    steps = len(x)
                except TypeError:
                    raise ValueError("steps_per_epoch is required for infinite datasets")
        else:
            xt, yt = self._prep_xy(x, y)
            if validation_split and validation_data is None:
                cut = int(len(xt) * (1 - validation_split))
                validation_data = (xt[cut:], yt[cut:])
                xt, yt = xt[:cut], yt[:cut]
            samples = len(xt)
            steps = steps_per_epoch or int(math.ceil(samples / batch_size))
        self.history = cbks.History()
        cb_list = [cbks.Callback()] + list(callbacks or []) + [self.history]
        if verbose:
            cb_list.append(cbks.ProgbarLogger(verbose))
        params = {"batch_size": batch_size, "epochs": epochs, "steps": steps, "samples": samples,
                  "verbose": verbose, "do_validation": validation_data is not None,
                  "metrics": list(self.metrics_names)}
        cb = cbks.CallbackList(cb_list, self, params)
        self.stop_training = False
        cb.on_train_begin({})
        for epoch in range(initial_epoch, epochs):
            self.train()
            cb.on_epoch_begin(epoch, {})
            sums: Dict[str, float] = {}
            seen = 0
            if dataset:
                batches = (self._prep_xy(*next(it)) for _ in range(steps))
            else:
                batches = self._batches(xt, yt, batch_size, shuffle)
            for b, (xb, yb) in enumerate(batches):
                if b >= steps:
                    break
                logs = {"batch": b, "size": int(xb.shape[0])}
                cb.on_train_batch_begin(b, logs)
                loss, mets = self._train_step(xb, yb)
                vals = {"loss": loss, **mets}
                host = {k: float(v) for k, v in vals.items()}
                logs.update(host)
                n = int(xb.shape[0])
                for k, v in host.items():
                    sums[k] = sums.get(k, 0.0) + v * n
                seen += n
                cb.on_train_batch_end(b, logs)
                if self.stop_training:
                    break
            epoch_logs = {k: v / max(seen, 1) for k, v in sums.items()}
            if validation_data is not None:
                vx, vy = validation_data[0], validation_data[1]
                vres = self.evaluate(vx, vy, batch_size=batch_size or 32, verbose=0,
                                     steps=validation_steps)
                vres = vres if isinstance(vres, list) else [vres]
                for nm, v in zip(self.metrics_names, vres):
                    epoch_logs["val_" + nm] = v
            cb.on_epoch_end(epoch, epoch_logs)
            if self.stop_training:
                break
        cb.on_train_end({})
        return self.history

    @torch.no_grad()
    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, steps=None, **kw):
        self.eval()
        sums: Dict[str, float] = {}
        seen = 0
        if self._is_dataset(x):
            it = iter(x)
            batches = ((self._prep_xy(*next(it))) for _ in range(steps or len(x)))
        else:
            xt, yt = self._prep_xy(x, y)
            batches = self._batches(xt, yt, batch_size or 32, False)
        for xb, yb in batches:
            out, logits = self._forward(xb, False)
            vals = {"loss": self._loss_value(yb, out, logits), **self._metric_values(yb, out)}
            n = int(xb.shape[0])
            for k, v in vals.items():
                sums[k] = sums.get(k, 0.0) + float(v) * n
            seen += n
        res = [sums.get(k, 0.0) / max(seen, 1) for k in self.metrics_names]
        if verbose:
            print(" - ".join(f"{k}: {v:.4f}" for k, v in zip(self.metrics_names, res)))
        return res if len(res) > 1 else res[0]

    @torch.no_grad()
    def predict(self, x, batch_size=32, verbose=0, **kw):
        self.eval()
        xt = _to_tensor(x, self.device_, torch.float32)
        outs = [self._forward(xt[i:i + batch_size], False)[0].float().cpu()
                for i in range(0, len(xt), batch_size)]
        return torch.cat(outs).numpy()

    def train_on_batch(self, x, y):
        self.train()
        xt, yt = self._prep_xy(x, y)
        loss, mets = self._train_step(xt, yt)
        res = [float(loss)] + [float(v) for v in mets.values()]
        return res if len(res) > 1 else res[0]

    # -- persistence ----------------------------------------------------------
    def get_config(self):
        raise NotImplementedError

    def _state_tensors(self, include_optimizer=True):
        t = {f"weights/{k}": v.detach().contiguous().cpu() for k, v in self.state_dict().items()}
        if include_optimizer and self.optimizer is not None and self.optimizer._impl is not None:
            impl = self.optimizer._impl
            pidx = {id(p): i for i, p in enumerate(self.optimizer._params)}
            for p, st in impl.state.items():
                for k, v in st.items():
                    if torch.is_tensor(v) and v.dim() > 0:
                        t[f"optimizer/{pidx[id(p)]}/{k}"] = v.detach().contiguous().float().cpu()
        return t

    def save(self, filepath, overwrite=True, include_optimizer=True):
        from safetensors.torch import save_file
        meta = {"format": "mivod.kerasfw/1", "model_config": json.dumps(self.get_config())}
        if self.optimizer is not None:
            meta["optimizer_config"] = json.dumps(O.serialize(self.optimizer))
            meta["optimizer_iterations"] = str(self.optimizer.iterations)
            meta["training_config"] = json.dumps({
                "loss": self.loss if isinstance(self.loss, str) else LS.name_of(self.loss),
                "loss_from_logits": bool(getattr(self.loss, "from_logits", False)),
                "metrics": [m for m in self._metric_specs if isinstance(m, str)]})
        save_file(self._state_tensors(include_optimizer), filepath, metadata=meta)

    def save_weights(self, filepath):
        from safetensors.torch import save_file
        save_file(self._state_tensors(False), filepath, metadata={"format": "mivod.kerasfw/1"})

    def load_weights(self, filepath):
        from safetensors.torch import load_file
        t = load_file(filepath)
        sd = {k[len("weights/"):]: v for k, v in t.items() if k.startswith("weights/")}
        self.load_state_dict(sd)

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        print_fn("_" * 65)
        print_fn(f"{'Layer (type)':<30}{'Output Shape':<22}{'Param #':>10}")
        print_fn("=" * 65)
        shape = getattr(self, "_input_shape", None)
        for lyr in self._keras_layers():
            if shape is not None:
                shape = lyr.compute_output_shape(shape)
            print_fn(f"{lyr.name + ' (' + type(lyr).__name__ + ')':<30}"
                     f"{str((None,) + tuple(shape)) if shape is not None else '?':<22}"
                     f"{lyr.count_params():>10,}")
        print_fn("=" * 65)
        print_fn(f"Total params: {self.count_params():,}")


class Sequential(Model):
    def __init__(self, layers=None, name=None):
        super().__init__(name=name or L._uid("sequential"))
        self.seq = nn.ModuleList()
        self._input_shape = None
        for lyr in layers or []:
            self.add(lyr)

    def add(self, layer: L.Layer):
        if not isinstance(layer, L.Layer):
            raise TypeError("Sequential.add expects a mivod.kerasfw layer")
        if not self.seq and layer.input_shape_arg is not None:
            self._input_shape = tuple(layer.input_shape_arg)
        self.seq.append(layer)
        if self._input_shape is not None:
            self._build_shapes()

    def _build_shapes(self):
        s = self._input_shape
        for lyr in self.seq:
            if not lyr.built:
                lyr.build(s)
            s = lyr.compute_output_shape(s)
        self.output_shape = (None,) + tuple(s)

    def build(self, input_shape):
        self._input_shape = tuple(input_shape[1:]) if len(input_shape) and input_shape[0] is None \
            else tuple(input_shape)
        self._build_shapes()
        self.to(self.device_)

    def _ensure_built(self, x):
        if self._input_shape is None or not all(l.built for l in self.seq):
            self._input_shape = tuple(x.shape[1:])
            self._build_shapes()
            self.to(x.device)
            if self.optimizer is not None and self.optimizer._impl is not None:
                raise RuntimeError("model was built after the optimizer started")

    def _forward(self, x, training):
        self._ensure_built(x)
        n = len(self.seq)
        logits = None
        for i, lyr in enumerate(self.seq):
            last = i == n - 1
            if last and getattr(lyr, "activation_name", None) == "softmax" and \
                    isinstance(lyr, (L.Dense, L.Activation)):
                if isinstance(lyr, L.Dense):
                    w = lyr.weight if lyr.weight.dtype == x.dtype else lyr.weight.to(x.dtype)
                    b = lyr.bias
                    logits = F.linear(x, w, None if b is None else b.to(x.dtype))
                else:
                    logits = x
                x = torch.softmax(logits, dim=-1)
            else:
                x = lyr(x, training=training)
        return x, logits

    @property
    def input_shape(self):
        return (None,) + tuple(self._input_shape) if self._input_shape else None

    def get_config(self):
        return {"class_name": "Sequential", "name": self.name,
                "input_shape": list(self._input_shape) if self._input_shape else None,
                "layers": [{"class_name": type(l).__name__, "config": l.get_config()}
                           for l in self.seq]}

    @classmethod
    def from_config(cls, cfg, custom_objects=None):
        custom_objects = custom_objects or {}
        m = cls(name=cfg.get("name"))
        for lc in cfg["layers"]:
            lcls = custom_objects.get(lc["class_name"]) or L.LAYERS[lc["class_name"]]
            c = dict(lc["config"])
            c.pop("trainable", None)
            m.seq.append(lcls(**c))
        if cfg.get("input_shape"):
            m._input_shape = tuple(cfg["input_shape"])
            m._build_shapes()
        return m


def load_model(filepath, custom_objects=None, compile=True):
    """Rebuild a model saved by ``Model.save`` (architecture, weights,
    optimizer + its slot state).  ``custom_objects`` maps class names to
    classes (horovod's ``load_model`` uses it to re-wrap the optimizer)."""
    from safetensors import safe_open
    from safetensors.torch import load_file
    with safe_open(filepath, framework="pt") as f:
        meta = f.metadata() or {}
    if "model_config" not in meta:
        raise ValueError(f"{filepath} is not a mivod.kerasfw model file")
    cfg = json.loads(meta["model_config"])
    if cfg.get("class_name") != "Sequential":
        raise ValueError("only Sequential models can be rebuilt from config")
    model = Sequential.from_config(cfg, custom_objects)
    tensors = load_file(filepath)
    sd = {k[len("weights/"):]: v for k, v in tensors.items() if k.startswith("weights/")}
    if model._input_shape is None:
        raise ValueError("saved model has no input shape")
    model.to(model.device_)
    model.load_state_dict(sd)
    if compile and "optimizer_config" in meta:
        opt = O.deserialize(json.loads(meta["optimizer_config"]), custom_objects)
        tc = json.loads(meta.get("training_config", "{}"))
        loss = tc.get("loss")
        if tc.get("loss_from_logits") and loss in ("SparseCategoricalCrossentropy",
                                                   "CategoricalCrossentropy"):
            loss = getattr(LS, loss)(from_logits=True)
        elif loss in ("SparseCategoricalCrossentropy", "CategoricalCrossentropy",
                      "BinaryCrossentropy", "MeanSquaredError"):
            loss = getattr(LS, loss)()
        model.compile(optimizer=opt, loss=loss, metrics=tc.get("metrics"))
        opt.iterations = int(meta.get("optimizer_iterations", "0"))
        ost = {k: v for k, v in tensors.items() if k.startswith("optimizer/")}
        if ost:
            params = model.trainable_weights
            opt._params = params
            opt._impl = opt._make_impl(params)
            if hasattr(opt._impl, "_mv_build"):
                opt._impl._mv_build()
            with torch.no_grad():
                for k, v in ost.items():
                    _, i, name = k.split("/", 2)
                    p = params[int(i)]
                    st = opt._impl.state[p]
                    if name in st and torch.is_tensor(st[name]):
                        st[name].copy_(v.to(st[name].device))
                    else:
                        st[name] = v.to(p.device)
            if hasattr(opt._impl, "_mv_arenas"):
                for a in opt._impl._mv_arenas or []:
                    a.step = opt.iterations
    return model
