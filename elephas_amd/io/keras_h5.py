"""Keras HDF5 model format (tf.keras <= 2.11 ``.h5``/``.keras`` layout).

Layout written (keras/saving/legacy/hdf5_format.py conventions):
  /                       attrs: keras_version, backend, model_config (JSON),
                                 training_config (JSON, when compiled)
  /model_weights          attrs: layer_names, backend, keras_version
  /model_weights/<layer>  attrs: weight_names  (e.g. b'dense/kernel:0')
  /model_weights/<layer>/<layer>/kernel:0, bias:0   fp32 datasets
  /optimizer_weights      attrs: weight_names ('<opt>/iter:0', '<opt>/<layer>/kernel/<slot>:0', ...)
                          datasets at those paths (written when the model has trained and
                          so owns optimizer state; restored into its trainer on load)
Attributes Keras split into numbered chunks because they exceeded the 64 KiB
object-header limit (``layer_names0``, ``layer_names1``, ...) are joined on read
(keras hdf5_format.load_attributes_from_hdf5_group).
Elephas adds ``distributed_config`` to the root attributes
(reference elephas/spark_model.py:117-125) through ``h5lite.File(..., 'a')``.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np

from . import h5lite
from ..models import optimizers as O


def _s(v) -> str:
    if isinstance(v, bytes):
        return v.decode("utf-8")
    if isinstance(v, np.ndarray) and v.shape == ():
        v = v[()]
    if isinstance(v, (bytes, np.bytes_)):
        return bytes(v).decode("utf-8")
    return str(v)


def _training_config(model) -> Optional[dict]:
    if not getattr(model, "_compiled", False) or getattr(model, "_compiled_for_predict_only", False):
        return None
    loss = model.loss if isinstance(model.loss, str) else getattr(model.loss, "__name__", str(model.loss))
    metrics = [m if isinstance(m, str) else getattr(m, "__name__", str(m)) for m in model.compiled_metrics._metrics]
    return {"loss": loss, "metrics": metrics, "weighted_metrics": None, "loss_weights": None,
            "optimizer_config": O.serialize(model.optimizer)}


def _get_attr(group, name, default=None):
    """Attribute ``name``, or the concatenation of its Keras chunks name0, name1, ..."""
    if name in group.attrs:
        return group.attrs[name]
    parts, i = [], 0
    while f"{name}{i}" in group.attrs:
        parts.append(np.atleast_1d(group.attrs[f"{name}{i}"]))
        i += 1
    if not parts:
        return default
    return np.concatenate(parts)


def _var_specs(model):
    """(Keras variable name, shape) of every weight in get_weights() order."""
    out = []
    for l in model._layers:
        for i, w in enumerate(l.get_weights()):
            out.append((f"{l.name}/{'kernel' if i == 0 else 'bias'}", np.shape(w)))
    return out


def _write_optimizer(f, model):
    opt = getattr(model, "optimizer", None)
    trainers = getattr(model, "_trainers", None) or {}
    if opt is None or not trainers:
        return  # never trained: Keras writes no optimizer weights either
    t = next(iter(trainers.values()))
    try:
        state, iters = t.get_state_flat()
    except Exception:  # noqa: BLE001 - an engine without exportable state
        return
    slots = opt.slot_names()
    name = getattr(opt, "_name", type(opt).__name__)
    names = [f"{name}/iter:0"]
    vals = [np.asarray(int(np.asarray(iters).reshape(-1)[0]), np.int64)]
    specs = _var_specs(model)
    st = np.asarray(state)[0]
    for si, slot in enumerate(slots):
        if si >= st.shape[0]:
            break
        off = 0
        for vname, shape in specs:
            n = int(np.prod(shape))
            names.append(f"{name}/{vname}/{slot}:0")
            vals.append(np.asarray(st[si, off:off + n], np.float32).reshape(shape))
            off += n
    g = f.create_group("optimizer_weights")
    g.attrs["weight_names"] = names
    for n, v in zip(names, vals):
        g.create_dataset(n, data=v)


def _read_optimizer(f, model):
    """optimizer_weights -> (state [planes, n_params], iterations), applied to the
    model's trainer when it is created (models.training.Model._trainer)."""
    if "optimizer_weights" not in f or getattr(model, "optimizer", None) is None:
        return
    g = f["optimizer_weights"]
    names = [_s(n) for n in np.atleast_1d(_get_attr(g, "weight_names", np.zeros(0, "S1")))]
    by = {}
    for n in names:
        try:
            by[n] = g[n][()]
        except KeyError:
            continue
    opt = model.optimizer
    oname = getattr(opt, "_name", type(opt).__name__)
    it = by.get(f"{oname}/iter:0")
    slots = opt.slot_names()
    specs = _var_specs(model)
    total = sum(int(np.prod(s)) for _, s in specs)
    state = np.zeros((max(opt.n_state(), 1), total), np.float32)
    if "state_init" in (opt.native() or (0, {}, 0))[1]:
        state[:] = float(opt.native()[1]["state_init"])
    found = it is not None
    for si, slot in enumerate(slots):
        off = 0
        for vname, shape in specs:
            n = int(np.prod(shape))
            v = by.get(f"{oname}/{vname}/{slot}:0")
            if v is not None:
                state[si, off:off + n] = np.asarray(v, np.float32).reshape(-1)
                found = True
            off += n
    if found:
        model._pending_optimizer_state = (state, int(it) if it is not None else 0)


def _write_weights(group, model):
    from ..models.training import KERAS_VERSION, BACKEND
    layers = [l for l in model._layers]
    group.attrs["layer_names"] = [l.name for l in layers]
    group.attrs["backend"] = BACKEND
    group.attrs["keras_version"] = KERAS_VERSION
    for l in layers:
        g = group.create_group(l.name)
        ws = l.get_weights()
        names = []
        if ws:
            names.append(f"{l.name}/kernel:0")
            if len(ws) > 1:
                names.append(f"{l.name}/bias:0")
        g.attrs["weight_names"] = names
        for n, w in zip(names, ws):
            g.create_dataset(n, data=np.asarray(w, np.float32))


def save_model(model, filepath, overwrite: bool = True, include_optimizer: bool = True) -> None:
    from ..models.training import KERAS_VERSION, BACKEND
    filepath = str(filepath)
    if os.path.exists(filepath) and not overwrite:
        raise FileExistsError(filepath)
    f = h5lite.File(filepath, "w")
    f.attrs["backend"] = BACKEND
    f.attrs["keras_version"] = KERAS_VERSION
    f.attrs["model_config"] = model.to_json()
    tc = _training_config(model) if include_optimizer else None
    if tc is not None:
        f.attrs["training_config"] = json.dumps(tc)
    _write_weights(f.create_group("model_weights"), model)
    if tc is not None:
        _write_optimizer(f, model)
    f.close()


def _read_weights(group, model):
    names = [_s(n) for n in np.atleast_1d(_get_attr(group, "layer_names"))]
    by_name = {l.name: l for l in model._layers}
    for ln in names:
        if ln not in by_name:
            raise ValueError(f"layer {ln} in file is not in the model")
        g = group[ln]
        wn = [_s(n) for n in np.atleast_1d(_get_attr(g, "weight_names", np.zeros(0, "S1")))]
        wn = [n for n in wn if n]
        if wn:
            by_name[ln].set_weights([g[n][()] for n in wn])


def load_model(filepath, custom_objects=None, compile: bool = True):
    from ..models.training import model_from_json
    f = h5lite.File(str(filepath), "r")
    model = model_from_json(_s(f.attrs["model_config"]), custom_objects)
    _read_weights(f["model_weights"], model)
    tc = f.attrs.get("training_config")
    if compile and tc is not None:
        cfg = json.loads(_s(tc))
        opt = O.deserialize(cfg["optimizer_config"], custom_objects)
        loss = cfg["loss"]
        if custom_objects and isinstance(loss, str) and loss in custom_objects:
            loss = custom_objects[loss]
        model.compile(optimizer=opt, loss=loss, metrics=cfg.get("metrics") or [], custom_objects=custom_objects)
        _read_optimizer(f, model)
    return model


def save_weights(model, filepath):
    f = h5lite.File(str(filepath), "w")
    _write_weights(f, model)
    f.close()


def load_weights(model, filepath):
    f = h5lite.File(str(filepath), "r")
    g = f["model_weights"] if "model_weights" in f else f
    _read_weights(g, model)
