"""Model export (tf.contrib.session_bundle.exporter equivalent).

Reference (model_export.py:50-66):
    exporter.Exporter(saver).init(graph_def, named_graph_signatures={
        'inputs': generic_signature({'x': x}), 'outputs': generic_signature({'y': y_pred})})
    .export('./model/', tf.constant('0003'), sess)
which writes `./model/00000003/{export.meta, export-00000-of-00001}`.

Here: `<base>/<%08d version>/` holds a TF V2 bundle with prefix `export`
(`export.index`, `export.data-00000-of-00001`, readable by
tf.train.NewCheckpointReader) and `export.meta.json` -- the signatures
(name -> tensor name, shape, dtype), the variable list and a serving
recipe.  The directory is built under a temp name and renamed, like the
original, so a reader never sees a partial export.  `load_session_bundle`
returns the restored tensors + signatures; for graphs made of the standard
layers a `predict` function is rebuilt from the recipe (linear / MLP).
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from .graph import Tensor, get_default_graph
from .saver import Saver, read_bundle_index, read_tensor

VERSION_FORMAT = "%08d"


def generic_signature(name_tensor_map: Dict[str, Tensor]) -> Dict[str, Any]:
    return {"kind": "generic", "map": {k: v for k, v in name_tensor_map.items()}}


def regression_signature(input_tensor, output_tensor) -> Dict[str, Any]:
    return {"kind": "regression", "map": {"input": input_tensor, "output": output_tensor}}


def classification_signature(input_tensor, classes_tensor=None, scores_tensor=None) -> Dict[str, Any]:
    m = {"input": input_tensor}
    if classes_tensor is not None:
        m["classes"] = classes_tensor
    if scores_tensor is not None:
        m["scores"] = scores_tensor
    return {"kind": "classification", "map": m}


def _desc(t) -> Dict[str, Any]:
    return {"name": getattr(t, "name", str(t)), "shape": list(t.shape) if getattr(t, "shape", None) else None,
            "dtype": str(getattr(t, "dtype", None))}


class Exporter:
    def __init__(self, saver: Optional[Saver] = None):
        self.saver = saver or Saver()
        self.graph_def = None
        self.named = {}
        self.default = None
        self.serving_recipe = None

    def init(self, graph_def=None, init_op=None, clear_devices=False, default_graph_signature=None,
             named_graph_signatures=None, assets_collection=None, assets_callback=None,
             serving_recipe: Optional[Dict[str, Any]] = None):
        self.graph_def = graph_def
        self.named = dict(named_graph_signatures or {})
        self.default = default_graph_signature
        self.serving_recipe = serving_recipe
        return self

    def export(self, export_dir_base: str, global_step_tensor, sess, exports_to_keep=None) -> str:
        v = global_step_tensor
        if isinstance(v, Tensor):
            v = sess.run(v)
        if isinstance(v, (bytes, np.bytes_)):
            v = v.decode()
        version = int(np.asarray(v).item()) if not isinstance(v, str) else int(v)
        final = os.path.join(export_dir_base, VERSION_FORMAT % version)
        tmp = os.path.join(export_dir_base, "temp-" + VERSION_FORMAT % version)
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp)
        self.saver.save(sess, os.path.join(tmp, "export"), write_state=False, write_meta_graph=False)
        meta = {
            "format": "dtf-session-bundle-v1",
            "version": version,
            "signatures": {name: {"kind": s["kind"], "map": {k: _desc(t) for k, t in s["map"].items()}}
                           for name, s in self.named.items()},
            "default_signature": None if self.default is None else
            {"kind": self.default["kind"], "map": {k: _desc(t) for k, t in self.default["map"].items()}},
            "variables": {n: {"shape": list(e["shape"]), "dtype": int(e["dtype"])}
                          for n, e in read_bundle_index(os.path.join(tmp, "export")).items() if n},
            "graph_def": self.graph_def.decode() if isinstance(self.graph_def, bytes) else self.graph_def,
            "serving_recipe": self.serving_recipe,
        }
        with open(os.path.join(tmp, "export.meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        shutil.rmtree(final, ignore_errors=True)
        os.rename(tmp, final)
        if exports_to_keep:
            vers = sorted(d for d in os.listdir(export_dir_base) if d.isdigit())
            for d in vers[:-exports_to_keep]:
                shutil.rmtree(os.path.join(export_dir_base, d), ignore_errors=True)
        return final


class SessionBundle:
    def __init__(self, path: str, meta: Dict[str, Any], tensors: Dict[str, torch.Tensor]):
        self.path, self.meta, self.tensors = path, meta, tensors
        self.signatures = meta["signatures"]
        self.predict: Optional[Callable] = _build_predict(meta.get("serving_recipe"), tensors)


def _build_predict(recipe, t):
    """Rebuild a forward function from a serving recipe, e.g.
    {"type": "linear", "w": "test/weights", "b": "test/bias"} or
    {"type": "mlp", "layers": [[w, b, act], ...], "output": "softmax"}."""
    if not recipe:
        return None
    if recipe["type"] == "linear":
        w, b = t[recipe["w"]].float(), t[recipe["b"]].float()
        return lambda x: torch.as_tensor(np.asarray(x, np.float32)) @ w + b
    if recipe["type"] == "mlp":
        acts = {"sigmoid": torch.sigmoid, "relu": torch.relu, "none": lambda z: z, None: lambda z: z}
        layers = [(t[w].float(), t[b].float(), acts[a]) for w, b, a in recipe["layers"]]

        def f(x):
            h = torch.as_tensor(np.asarray(x, np.float32))
            for w, b, a in layers:
                h = a(h @ w + b)
            return torch.softmax(h, 1) if recipe.get("output") == "softmax" else h
        return f
    raise ValueError(f"unknown serving recipe {recipe['type']}")


def load_session_bundle(export_dir: str) -> SessionBundle:
    with open(os.path.join(export_dir, "export.meta.json")) as f:
        meta = json.load(f)
    prefix = os.path.join(export_dir, "export")
    tensors = {n: read_tensor(prefix, n) for n in read_bundle_index(prefix) if n}
    return SessionBundle(export_dir, meta, tensors)


def graph_def():
    return get_default_graph().as_graph_def()
