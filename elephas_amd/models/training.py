"""Keras-compatible ``Model`` / ``Sequential`` with compile/fit/evaluate/predict.

Reproduces the tf.keras 2.10 surface the reference relies on
(``get_weights`` order, ``to_json``/``model_from_json``,
``compile``, ``fit(... validation_split)`` -> ``History``, ``train_on_batch``,
``predict``, ``evaluate`` -> scalar or ``[loss, *metrics]``, ``save``).
Execution goes to the native MI355X executor or the torch engine
(``elephas_amd/ops/engine.py``).
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import losses as L
from . import metrics as M
from . import optimizers as O
from .layers import (Dense, InputLayer, KerasTensor, Layer, deserialize as deserialize_layer,
                     serialize as serialize_layer, unique_name)

KERAS_VERSION = "2.10.0"
BACKEND = "tensorflow"  # config-compatibility tag only: execution is HIP/torch


class History:
    def __init__(self):
        self.history: Dict[str, list] = {}
        self.epoch: List[int] = []
        self.params: dict = {}
        self.model = None


class _CompiledMetrics:
    def __init__(self, metrics):
        self._metrics = list(metrics) if metrics is not None else []


class Model:
    """Functional model over a chain of single-input layers."""

    def __init__(self, inputs=None, outputs=None, name: Optional[str] = None):
        self.name = name or unique_name("model")
        self._layers: List[Layer] = []
        self._compiled = False
        self._trainers = {}
        self.optimizer = None
        self.stop_training = False
        if inputs is not None:
            self._init_graph(inputs, outputs)

    # ----------------------------------------------------------------- graph
    def _init_graph(self, inputs, outputs):
        ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
        if len(ins) != 1 or len(outs) != 1:
            raise NotImplementedError("only single-input single-output models are supported")
        chain = []
        layer = outs[0].layer
        while True:
            chain.append(layer)
            if isinstance(layer, InputLayer):
                break
            if len(layer.inbound) != 1:
                raise NotImplementedError(f"layer {layer.name} is not part of a simple chain")
            layer = layer.inbound[0]
        chain.reverse()
        if chain[0] is not ins[0].layer:
            raise ValueError("outputs are not connected to inputs")
        self._layers = chain
        self._input_layer = chain[0]

    @property
    def layers(self) -> List[Layer]:
        return list(self._layers)

    @property
    def input_shape(self):
        return self._layers[0]._batch_input_shape if self._layers else None

    @property
    def output_shape(self):
        return self._layers[-1].output_shape if self._layers else None

    @property
    def built(self) -> bool:
        return bool(self._layers) and all(l.built for l in self._layers)

    def get_layer(self, name=None, index=None):
        if index is not None:
            return self.layers[index]
        for l in self._layers:
            if l.name == name:
                return l
        raise ValueError(f"No such layer: {name}")

    # --------------------------------------------------------------- weights
    def get_weights(self) -> List[np.ndarray]:
        out = []
        for l in self._layers:
            out.extend(l.get_weights())
        return out

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        ws = list(weights)
        i = 0
        for l in self._layers:
            n = len(l.weights)
            if n:
                l.set_weights(ws[i:i + n])
                i += n
        if i != len(ws):
            raise ValueError(f"model expects {i} weight arrays, got {len(ws)}")

    @property
    def weights(self):
        return self.get_weights()

    @property
    def trainable_weights(self):
        return self.get_weights()

    def count_params(self) -> int:
        return int(sum(l.count_params() for l in self._layers))

    def summary(self, print_fn=print) -> None:
        print_fn(f'Model: "{self.name}"')
        print_fn(f"{'Layer (type)':<32}{'Output Shape':<24}{'Param #':>10}")
        for l in self._layers:
            print_fn(f"{l.name + ' (' + type(l).__name__ + ')':<32}{str(l.output_shape):<24}{l.count_params():>10}")
        print_fn(f"Total params: {self.count_params():,}")

    # ------------------------------------------------------------ serialize
    def _functional_config(self) -> dict:
        layers = []
        prev = None
        for l in self._layers:
            d = serialize_layer(l)
            d["name"] = l.name
            d["inbound_nodes"] = [] if prev is None else [[[prev.name, 0, 0, {}]]]
            layers.append(d)
            prev = l
        return {"name": self.name, "layers": layers,
                "input_layers": [[self._layers[0].name, 0, 0]],
                "output_layers": [[self._layers[-1].name, 0, 0]]}

    def get_config(self) -> dict:
        return self._functional_config()

    def _class_name(self) -> str:
        return "Functional"

    def to_json(self, **kwargs) -> str:
        return json.dumps({"class_name": self._class_name(), "config": self.get_config(),
                           "keras_version": KERAS_VERSION, "backend": BACKEND}, **kwargs)

    # --------------------------------------------------------------- compile
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, steps_per_execution=None, custom_objects=None, **kwargs):
        if loss is None:
            raise ValueError("compile() needs a loss")
        if not self.built:
            raise ValueError("build the model (give the first layer an input shape) before compile()")
        self.optimizer = O.get(optimizer)
        self.loss = loss
        self._loss_spec = L.get(loss, custom_objects)
        mets = metrics or []
        if isinstance(mets, dict):
            mets = list(mets.values())
        self.compiled_metrics = _CompiledMetrics(mets)
        n_out = int(self._layers[-1].output_shape[-1])
        self._metric_specs = [M.get(m, n_out, self._loss_spec, custom_objects) for m in mets]
        self.compiled_loss = self._loss_spec
        self._compiled = True
        self._trainers = {}

    @property
    def metrics_names(self) -> List[str]:
        if not self._compiled:
            return []
        return ["loss"] + [m.name for m in self._metric_specs]

    def _require_compiled(self):
        if not self._compiled:
            raise RuntimeError("You must compile your model before training/testing. Use `model.compile(optimizer, loss)`.")

    # ---------------------------------------------------------------- engine
    def _trainer(self, batch_size: int):
        from ..ops.engine import make_trainer
        key = int(batch_size)
        from .layers import weight_epoch
        t = self._trainers.get(key)
        if t is None:
            t = make_trainer(self, 1, key)
            self._trainers = {key: t}  # one live trainer: it owns the optimizer state
            pending = getattr(self, "_pending_optimizer_state", None)
            if pending is not None:  # optimizer weights restored from an HDF5 checkpoint
                t.set_state_flat(pending[0][None], [pending[1]])
                self._pending_optimizer_state = None
        elif getattr(t, "_weight_epoch", None) != weight_epoch():
            # the host weights changed since the trainer last saw them (a repeated
            # predict / evaluate on unchanged weights skips this upload: 150 MB on Wide)
            from ..ops.plan import flatten_weights
            t.set_weights_flat(flatten_weights(self.get_weights()))
        t._weight_epoch = weight_epoch()
        return t

    def _pull(self, t):
        from ..ops.plan import unflatten_weights
        from .layers import weight_epoch
        self.set_weights(unflatten_weights(t.get_weights_flat()[0], self.get_weights()))
        t._weight_epoch = weight_epoch()  # host and device copies agree again

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None, validation_split=0.0,
            validation_data=None, shuffle=True, initial_epoch=0, **kwargs) -> History:
        self._require_compiled()
        bs = int(batch_size or 32)
        t = self._trainer(bs)
        x = np.asarray(x)
        y = np.asarray(y)
        t.set_data([x], [y], validation_split if validation_data is None else 0.0, shuffle=bool(shuffle))
        hist = t.fit(int(epochs) - int(initial_epoch), verbose=verbose if verbose else 0)[0] or {}
        self._pull(t)
        if validation_data is not None:
            vx, vy = validation_data[0], validation_data[1]
            res = t.evaluate(np.asarray(vx), np.asarray(vy), bs)
            hist["val_loss"] = [res[0]]
            for name, v in zip([m.name for m in self._metric_specs], res[1:]):
                hist["val_" + name] = [v]
        h = History()
        h.history = hist
        h.epoch = list(range(initial_epoch, int(epochs)))
        h.params = {"verbose": verbose, "epochs": epochs, "steps": None}
        h.model = self
        self.history = h
        return h

    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, return_dict=False, **kwargs):
        self._require_compiled()
        t = self._trainer(int(batch_size or 32))
        res = t.evaluate(np.asarray(x), np.asarray(y), batch_size)
        if return_dict:
            return dict(zip(self.metrics_names, res))
        return res if len(res) > 1 else res[0]

    def predict(self, x, batch_size=None, verbose=0, **kwargs) -> np.ndarray:
        if not self.built:
            raise ValueError("model is not built")
        if not self._compiled:
            # inference needs no loss; compile a throwaway configuration
            self._predict_only_compile()
        t = self._trainer(int(batch_size or 32))
        return t.predict(np.asarray(x), batch_size)

    def _predict_only_compile(self):
        n_out = int(self._layers[-1].output_shape[-1])
        self.optimizer = O.SGD()
        self._loss_spec = L.get("mean_squared_error")
        self._metric_specs = []
        self.compiled_metrics = _CompiledMetrics([])
        self._compiled = True
        self._compiled_for_predict_only = True
        _ = n_out

    def train_on_batch(self, x, y, **kwargs):
        self._require_compiled()
        x = np.asarray(x)
        t = self._trainer(len(x))
        res = t.train_on_batch(x, np.asarray(y))
        self._pull(t)
        return res if len(res) > 1 else res[0]

    def test_on_batch(self, x, y, **kwargs):
        return self.evaluate(x, y, batch_size=len(x), verbose=0)

    def predict_on_batch(self, x):
        return self.predict(x, batch_size=len(x))

    def __call__(self, x):
        return self.predict(x)

    # ----------------------------------------------------------------- save
    def save(self, filepath, overwrite=True, include_optimizer=True, save_format=None, **kwargs):
        from ..io.keras_h5 import save_model
        save_model(self, filepath, overwrite=overwrite, include_optimizer=include_optimizer)

    def save_weights(self, filepath, overwrite=True):
        from ..io.keras_h5 import save_weights
        save_weights(self, filepath)

    def load_weights(self, filepath):
        from ..io.keras_h5 import load_weights
        load_weights(self, filepath)


class Sequential(Model):
    def __init__(self, layers=None, name: Optional[str] = None):
        super().__init__(name=name or unique_name("sequential"))
        self._user_layers: List[Layer] = []
        for l in layers or []:
            self.add(l)

    def add(self, layer: Layer) -> None:
        if isinstance(layer, InputLayer):
            if self._user_layers:
                raise ValueError("InputLayer must be the first layer")
            self._layers = [layer]
            return
        if isinstance(layer, KerasTensor):
            raise TypeError("add() expects a layer")
        if not self._layers:
            if layer._batch_input_shape is not None:
                inp = InputLayer(batch_input_shape=layer._batch_input_shape, name=layer.name + "_input")
                self._layers = [inp]
        if self._layers:
            prev_shape = self._layers[-1].output_shape
            if not layer.built:
                layer.build(prev_shape)
            elif layer.input_shape is not None and prev_shape is not None and \
                    tuple(layer.input_shape[1:]) != tuple(prev_shape[1:]):
                raise ValueError(f"incompatible input shape for {layer.name}")
        self._layers.append(layer)
        self._user_layers.append(layer)
        self._trainers = {}

    def build(self, input_shape=None) -> None:
        if input_shape is None:
            return
        input_shape = tuple(input_shape)
        if input_shape and input_shape[0] is not None and len(input_shape) == 1:
            input_shape = (None,) + input_shape
        if not self._layers or not isinstance(self._layers[0], InputLayer):
            self._layers = [InputLayer(batch_input_shape=input_shape, name=unique_name("input"))] + \
                           [l for l in self._layers if not isinstance(l, InputLayer)]
        prev = self._layers[0].output_shape
        for l in self._layers[1:]:
            if not l.built:
                l.build(prev)
            prev = l.output_shape

    @property
    def layers(self):
        return [l for l in self._layers if not isinstance(l, InputLayer)]

    @property
    def built(self):
        return bool(self._layers) and isinstance(self._layers[0], InputLayer) and all(l.built for l in self._layers)

    def get_config(self) -> dict:
        layers = []
        for l in self._layers:
            layers.append(serialize_layer(l))
        return {"name": self.name, "layers": layers}

    def _class_name(self) -> str:
        return "Sequential"


# ------------------------------------------------------------ (de)serialization
def model_from_config(config: dict, custom_objects=None) -> Model:
    cls = config["class_name"]
    cfg = config["config"]
    if cls == "Sequential":
        m = Sequential(name=cfg.get("name"))
        for ld in cfg["layers"]:
            m.add(deserialize_layer(ld, custom_objects))
        return m
    if cls in ("Functional", "Model"):
        by_name = {}
        for ld in cfg["layers"]:
            by_name[ld["name"]] = (deserialize_layer(ld, custom_objects), ld.get("inbound_nodes", []))
        tensors = {}
        from .layers import KerasTensor as KT

        def tensor_of(name):
            if name in tensors:
                return tensors[name]
            layer, inbound = by_name[name]
            if isinstance(layer, InputLayer):
                t = KT(layer._batch_input_shape, layer)
            else:
                src = inbound[0][0][0]
                t = layer(tensor_of(src))
            tensors[name] = t
            return t

        inp = tensor_of(cfg["input_layers"][0][0])
        out = tensor_of(cfg["output_layers"][0][0])
        return Model(inputs=inp, outputs=out, name=cfg.get("name"))
    raise ValueError(f"Unknown model class {cls}")


def model_from_json(json_string: str, custom_objects=None) -> Model:
    return model_from_config(json.loads(json_string), custom_objects)


def clone_model(model: Model, custom_objects=None) -> Model:
    m = model_from_json(model.to_json(), custom_objects)
    m.set_weights(model.get_weights())
    return m
