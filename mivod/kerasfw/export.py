"""Serving export — the replacement for the reference's TF1 SavedModel export
(/root/reference/mnist_keras.py:116-140: predict signature ``input -> prob``,
SERVING tag, timestamped directory).

Writes ``<export_dir>/<YYYYmmdd-HHMMSS>/`` with ``model.safetensors`` (weights +
architecture metadata, loadable by ``mivod.kerasfw.load_model``) and
``signature.json`` describing the default serving signature.
"""
from __future__ import annotations

import json
import os
import time


def export_serving(model, export_dir: str, input_name: str = "input",
                   output_name: str = "prob", timestamp: bool = True) -> str:
    d = os.path.join(export_dir, time.strftime("%Y%m%d-%H%M%S")) if timestamp else export_dir
    os.makedirs(d, exist_ok=True)
    model.save(os.path.join(d, "model.safetensors"), include_optimizer=False)
    ishape = [-1] + list(model.input_shape[1:]) if getattr(model, "input_shape", None) else None
    oshape = [-1] + list(model.output_shape[1:]) if getattr(model, "output_shape", None) else None
    sig = {"tags": ["serve"], "signature_def": {"serving_default": {
        "inputs": {input_name: {"dtype": "float32", "shape": ishape}},
        "outputs": {output_name: {"dtype": "float32", "shape": oshape}},
        "method_name": "predict"}}}
    with open(os.path.join(d, "signature.json"), "w") as f:
        json.dump(sig, f, indent=2)
    return d


def load_serving(path: str):
    """(model, signature) from an export directory; ``model.predict`` serves it."""
    from .models import load_model
    model = load_model(os.path.join(path, "model.safetensors"), compile=False)
    with open(os.path.join(path, "signature.json")) as f:
        return model, json.load(f)
