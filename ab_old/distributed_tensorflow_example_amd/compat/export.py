"""Model export in the session_bundle layout (tf.contrib.session_bundle.exporter,
SURVEY N7/C26).

Reference (model_export.py:53-66):
    exporter.Exporter(saver).init(graph_def, named_graph_signatures={
        'inputs': generic_signature({'x': x}), 'outputs': generic_signature({'y': y_pred})})
    .export('./model/', tf.constant('0003'), sess)
which writes `./model/00000003/`: `export.meta` (a serialized MetaGraphDef),
the checkpoint (`export.index`, `export.data-00000-of-00001`) and the
`checkpoint` state file.

As in TF's exporter: `init` packs a `tensorflow.serving.Signatures` message
(default + named signatures; generic / regression / classification) into a
`google.protobuf.Any` and adds it to the graph collection
`serving_signatures` (and an init op to `serving_init_op`); `export` evaluates
the version tensor, refuses to overwrite an existing version, saves through
the Saver into `<dir>-tmp` with meta_graph_suffix "meta" -- so the MetaGraphDef
written next to the bundle carries the signatures -- renames it into place
and garbage-collects old versions (`exports_to_keep`).  Protos are encoded by
compat/meta_graph.py.

`load_session_bundle(export_dir)` is session_bundle.load_session_bundle_from_path:
it parses `export.meta`, rebuilds the graph from its GraphDef in a fresh
compat graph, restores the variables from the bundle and returns a session
plus the decoded meta graph; `bundle.predict(x)` runs the generic
`inputs`/`outputs` signatures the reference defines.
"""
from __future__ import annotations

import os
import shutil
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from . import meta_graph as M
from .graph import Graph, Tensor, get_default_graph
from .saver import Saver, read_bundle_index, read_tensor

VERSION_FORMAT = "%08d"            # session_bundle/constants.py VERSION_FORMAT_SPECIFIER
EXPORT_BASE_NAME = "export"
EXPORT_SUFFIX_NAME = "meta"
META_GRAPH_DEF_FILENAME = EXPORT_BASE_NAME + "." + EXPORT_SUFFIX_NAME


def generic_signature(name_tensor_map: Dict[str, Tensor]) -> Dict[str, Any]:
    return {"kind": "generic", "map": dict(name_tensor_map)}


def regression_signature(input_tensor, output_tensor) -> Dict[str, Any]:
    return {"kind": "regression", "map": {"input": input_tensor, "output": output_tensor}}


def classification_signature(input_tensor, classes_tensor=None, scores_tensor=None) -> Dict[str, Any]:
    m = {"input": input_tensor}
    if classes_tensor is not None:
        m["classes"] = classes_tensor
    if scores_tensor is not None:
        m["scores"] = scores_tensor
    return {"kind": "classification", "map": m}


def _version_of(v, sess) -> int:
    if isinstance(v, Tensor):
        v = sess.run(v)
    if isinstance(v, (bytes, np.bytes_)):
        v = v.decode()
    return int(v) if isinstance(v, str) else int(np.asarray(v).item())


class Exporter:
    def __init__(self, saver: Optional[Saver] = None):
        self.saver = saver or Saver()
        self._has_init = False
        self.graph_def = None

    def init(self, graph_def=None, init_op=None, clear_devices=False, default_graph_signature=None,
             named_graph_signatures=None, assets_collection=None, assets_callback=None):
        g = get_default_graph()
        self.graph_def = graph_def
        named = dict(named_graph_signatures or {})
        sig = M.signatures_proto(named, default_graph_signature)
        g.add_to_collection(M.SIGNATURES_KEY, M.AnyProto(M.SIGNATURES_TYPE_URL, sig))
        if init_op is not None:
            g.add_to_collection(M.INIT_OP_KEY, init_op)
        self._assets = list(assets_collection or [])
        self._assets_callback = assets_callback
        self._has_init = True
        return self

    def export(self, export_dir_base: str, global_step_tensor, sess, exports_to_keep=None) -> str:
        if not self._has_init:
            raise RuntimeError("init must be called first")
        version = _version_of(global_step_tensor, sess)
        final = os.path.join(export_dir_base, VERSION_FORMAT % version)
        if os.path.exists(final):
            raise RuntimeError(f"Overwriting exports can cause corruption and are not allowed. "
                               f"Duplicate export dir: {final}")
        tmp = final + "-tmp"
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp)
        self.saver.save(sess, os.path.join(tmp, EXPORT_BASE_NAME), meta_graph_suffix=EXPORT_SUFFIX_NAME)
        if self._assets:
            adir = os.path.join(tmp, "assets")
            os.makedirs(adir, exist_ok=True)
            for a in self._assets:
                src = a if isinstance(a, str) else sess.run(a)
                src = src.decode() if isinstance(src, bytes) else str(src)
                (self._assets_callback or shutil.copy)(src, os.path.join(adir, os.path.basename(src)))
        os.rename(tmp, final)
        if exports_to_keep:
            vers = sorted(d for d in os.listdir(export_dir_base) if d.isdigit())
            for d in vers[:-exports_to_keep]:
                shutil.rmtree(os.path.join(export_dir_base, d), ignore_errors=True)
        return final


class SessionBundle:
    """What load_session_bundle_from_path returns: (session, meta_graph_def),
    plus the decoded signatures and the restored tensors."""

    def __init__(self, path: str, session, meta_graph_def: Dict[str, Any], signatures: Dict[str, Any],
                 tensors: Dict[str, torch.Tensor]):
        self.path, self.session, self.meta_graph_def = path, session, meta_graph_def
        self.signatures = signatures["named_signatures"]
        self.default_signature = signatures["default_signature"]
        self.tensors = tensors
        self.predict: Optional[Callable] = self._generic_predict()

    def run(self, fetches, feed_dict=None):
        return self.session.run(fetches, feed_dict=feed_dict)

    def _generic_predict(self):
        ins, outs = self.signatures.get("inputs"), self.signatures.get("outputs")
        if not (ins and outs and ins["kind"] == outs["kind"] == "generic" and len(ins["map"]) == 1):
            return None
        x_name = next(iter(ins["map"].values()))
        y_names = list(outs["map"].values())

        def f(x):
            vals = self.session.run(y_names, feed_dict={x_name: np.asarray(x, np.float32)})
            return torch.as_tensor(vals[0]) if len(vals) == 1 else [torch.as_tensor(v) for v in vals]
        return f


def _variable_values(prefix: str, meta: Dict[str, Any]) -> Dict[str, torch.Tensor]:
    """Variable name -> value; partition variables (VariableDef with a
    SaveSliceInfoDef) get their slice of the full checkpoint tensor."""
    idx = read_bundle_index(prefix)
    out: Dict[str, torch.Tensor] = {}
    col = meta["collection_def"].get("variables", {"value": []})
    for raw in col["value"]:
        vd = M.parse_variable_def(raw)
        name = vd["variable_name"].split(":")[0]
        si = vd["save_slice_info_def"]
        if si is None:
            if name in idx:
                out[name] = read_tensor(prefix, name)
            continue
        full = read_tensor(prefix, si["full_name"])
        sl = tuple(slice(o, o + n) for o, n in zip(si["var_offset"], si["var_shape"]))
        out[name] = full[sl].clone()
    for name in idx:
        if name and name not in out and not any(k.startswith(name + "/part_") for k in out):
            out[name] = read_tensor(prefix, name)
    return out


def load_session_bundle(export_dir: str) -> SessionBundle:
    from .session import Session

    with open(os.path.join(export_dir, META_GRAPH_DEF_FILENAME), "rb") as f:
        meta = M.parse_meta_graph(f.read())
    col = meta["collection_def"].get(M.SIGNATURES_KEY)
    if not col or col["kind"] != "any_list" or len(col["value"]) != 1:
        raise RuntimeError(f"expected exactly one serving signatures entry in {export_dir}")
    anyv = col["value"][0]
    if anyv["type_url"] != M.SIGNATURES_TYPE_URL:
        raise RuntimeError(f"unexpected signatures type {anyv['type_url']}")
    sigs = M.parse_signatures(anyv["value"])
    prefix = os.path.join(export_dir, EXPORT_BASE_NAME)
    values = _variable_values(prefix, meta)
    g = Graph()
    with g.as_default():
        build = M.import_graph(meta["graph_def"], values)
        for s in list(sigs["named_signatures"].values()) + ([sigs["default_signature"]] if sigs["default_signature"] else []):
            for tname in s["map"].values():
                build(tname.split(":")[0])
        init = meta["collection_def"].get(M.INIT_OP_KEY)
    sess = Session(graph=g)
    if init and init["kind"] == "node_list":
        for op in init["value"]:
            try:
                with g.as_default():
                    sess.run(build(op))
            except NotImplementedError:
                pass
    tensors = {k: v for k, v in values.items()}
    for name in read_bundle_index(prefix):
        if name and name not in tensors:
            tensors[name] = read_tensor(prefix, name)
    return SessionBundle(export_dir, sess, meta, sigs, tensors)


load_session_bundle_from_path = load_session_bundle


def graph_def():
    return get_default_graph().as_graph_def()
