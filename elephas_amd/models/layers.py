"""Layers of the Keras-compatible model API.

The reference's models use exactly InputLayer/Input, Dense, Activation and
Dropout (reference tests/conftest.py:2-40, examples/*.py); configs serialise in
the tf.keras 2.10 ``to_json`` layout so ``model_from_json(model.to_json())``
round-trips (reference tests/test_ml_model.py:29-43).  Weights are held as fp32
numpy arrays in Keras order (kernel ``[in, out]``, bias ``[out]``).
"""
from __future__ import annotations

import re
from collections import defaultdict
from typing import List, Optional, Sequence

import numpy as np

from . import activations as A
from . import initializers as I

_name_counts = defaultdict(int)


def _snake(name: str) -> str:
    s = re.sub(r"(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", s).lower()


def unique_name(base: str) -> str:
    n = _name_counts[base]
    _name_counts[base] += 1
    return base if n == 0 else f"{base}_{n}"


def clear_session() -> None:
    _name_counts.clear()


class KerasTensor:
    """Symbolic tensor of the functional API: shape + producing layer."""

    def __init__(self, shape, layer: "Layer", node_index: int = 0, tensor_index: int = 0):
        self.shape = tuple(shape)
        self.layer = layer
        self.node_index = node_index
        self.tensor_index = tensor_index

    def __repr__(self):
        return f"<KerasTensor shape={self.shape} from {self.layer.name}>"


# Bumped whenever any layer attribute is (re)bound to an ndarray (build, set_weights,
# load): a model's device trainer re-uploads its weights only when this moved since
# its last sync (in-place edits of a weight array are not seen; use set_weights).
_WEIGHT_EPOCH = [0]


def weight_epoch() -> int:
    return _WEIGHT_EPOCH[0]


class Layer:
    def __setattr__(self, name, value):
        if isinstance(value, np.ndarray):
            _WEIGHT_EPOCH[0] += 1
        object.__setattr__(self, name, value)

    def __init__(self, name: Optional[str] = None, trainable: bool = True, dtype: str = "float32",
                 input_shape=None, batch_input_shape=None, input_dim=None, **kwargs):
        self.name = name or unique_name(_snake(type(self).__name__))
        self.trainable = trainable
        self.dtype = dtype
        self.built = False
        if input_dim is not None and input_shape is None:
            input_shape = (input_dim,)
        if batch_input_shape is not None:
            self._batch_input_shape = tuple(batch_input_shape)
        elif input_shape is not None:
            self._batch_input_shape = (None,) + tuple(input_shape)
        else:
            self._batch_input_shape = None
        self.inbound: List["Layer"] = []   # functional graph: producing layers
        self.input_shape = None
        self.output_shape = None

    # --- weights
    @property
    def weights(self) -> List[np.ndarray]:
        return []

    def get_weights(self) -> List[np.ndarray]:
        return [w.copy() for w in self.weights]

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        if len(weights) != 0:
            raise ValueError(f"Layer {self.name} has no weights")

    def count_params(self) -> int:
        return int(sum(w.size for w in self.weights))

    # --- shapes
    def build(self, input_shape) -> None:
        self.input_shape = tuple(input_shape)
        self.output_shape = self.compute_output_shape(input_shape)
        self.built = True

    def compute_output_shape(self, input_shape):
        return tuple(input_shape)

    # --- functional API
    def __call__(self, inputs):
        if isinstance(inputs, (list, tuple)):
            if len(inputs) != 1:
                raise NotImplementedError("multi-input layers are not supported")
            inputs = inputs[0]
        if not isinstance(inputs, KerasTensor):
            raise TypeError("layers are called on KerasTensors (functional API) in elephas_amd; "
                            "use Model.predict for eager inference")
        if not self.built:
            self.build(inputs.shape)
        self.inbound.append(inputs.layer)
        return KerasTensor(self.output_shape, self, node_index=len(self.inbound) - 1)

    # --- serialization
    def get_config(self) -> dict:
        cfg = {"name": self.name, "trainable": self.trainable, "dtype": self.dtype}
        if self._batch_input_shape is not None:
            cfg["batch_input_shape"] = list(self._batch_input_shape)
        return cfg

    @classmethod
    def from_config(cls, config: dict, custom_objects=None):
        return cls(**config)


class InputLayer(Layer):
    def __init__(self, input_shape=None, batch_size=None, dtype="float32", sparse=False, ragged=False,
                 name=None, batch_input_shape=None, **kwargs):
        if batch_input_shape is None and input_shape is not None:
            batch_input_shape = (batch_size,) + tuple(input_shape)
        if name is None:
            name = unique_name("input")
        super().__init__(name=name, dtype=dtype, batch_input_shape=batch_input_shape)
        self.sparse, self.ragged = sparse, ragged
        self.build(self._batch_input_shape)

    def get_config(self):
        return {"batch_input_shape": list(self._batch_input_shape), "dtype": self.dtype, "sparse": self.sparse,
                "ragged": self.ragged, "name": self.name}


def Input(shape=None, batch_size=None, name=None, dtype="float32", batch_shape=None, **kwargs) -> KerasTensor:
    if batch_shape is None:
        batch_shape = (batch_size,) + tuple(shape)
    layer = InputLayer(batch_input_shape=batch_shape, name=name, dtype=dtype)
    return KerasTensor(layer._batch_input_shape, layer)


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None,
                 activity_regularizer=None, kernel_constraint=None, bias_constraint=None,
                 custom_objects=None, **kwargs):
        super().__init__(**kwargs)
        self.units = int(units)
        self.activation = A.get(activation, custom_objects)
        self.use_bias = use_bias
        self.kernel_initializer = I.get(kernel_initializer)
        self.bias_initializer = I.get(bias_initializer)
        for reg in (kernel_regularizer, bias_regularizer, activity_regularizer, kernel_constraint, bias_constraint):
            if reg is not None:
                raise NotImplementedError("regularizers/constraints are not supported")
        self.kernel: Optional[np.ndarray] = None
        self.bias: Optional[np.ndarray] = None
        if self._batch_input_shape is not None:
            self.build(self._batch_input_shape)

    def build(self, input_shape):
        if self.built:
            return
        in_dim = int(input_shape[-1])
        self.kernel = np.asarray(self.kernel_initializer((in_dim, self.units)), dtype=np.float32)
        self.bias = np.asarray(self.bias_initializer((self.units,)), dtype=np.float32) if self.use_bias else None
        super().build(input_shape)

    def compute_output_shape(self, input_shape):
        return tuple(input_shape[:-1]) + (self.units,)

    @property
    def weights(self):
        if not self.built:
            return []
        return [self.kernel, self.bias] if self.use_bias else [self.kernel]

    def set_weights(self, weights):
        if not self.built:
            raise ValueError(f"Layer {self.name} is not built")
        ws = list(weights)
        exp = 2 if self.use_bias else 1
        if len(ws) != exp:
            raise ValueError(f"Layer {self.name} expects {exp} weight arrays, got {len(ws)}")
        k = np.asarray(ws[0], dtype=np.float32)
        if k.shape != self.kernel.shape:
            raise ValueError(f"kernel shape mismatch for {self.name}: {k.shape} vs {self.kernel.shape}")
        self.kernel = k.copy()
        if self.use_bias:
            b = np.asarray(ws[1], dtype=np.float32)
            if b.shape != self.bias.shape:
                raise ValueError(f"bias shape mismatch for {self.name}: {b.shape} vs {self.bias.shape}")
            self.bias = b.copy()

    def get_config(self):
        cfg = super().get_config()
        cfg.update({
            "units": self.units,
            "activation": A.serialize(self.activation),
            "use_bias": self.use_bias,
            "kernel_initializer": I.serialize(self.kernel_initializer),
            "bias_initializer": I.serialize(self.bias_initializer),
            "kernel_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
            "kernel_constraint": None, "bias_constraint": None,
        })
        return cfg

    @classmethod
    def from_config(cls, config, custom_objects=None):
        return cls(custom_objects=custom_objects, **config)


class Activation(Layer):
    def __init__(self, activation, custom_objects=None, **kwargs):
        super().__init__(**kwargs)
        self.activation = A.get(activation, custom_objects)
        if self._batch_input_shape is not None:
            self.build(self._batch_input_shape)

    def get_config(self):
        cfg = super().get_config()
        cfg["activation"] = A.serialize(self.activation)
        return cfg

    @classmethod
    def from_config(cls, config, custom_objects=None):
        return cls(custom_objects=custom_objects, **config)


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=None, **kwargs):
        super().__init__(**kwargs)
        if not 0.0 <= float(rate) < 1.0:
            raise ValueError(f"Dropout rate must be in [0, 1), got {rate}")
        if noise_shape is not None:
            raise NotImplementedError("Dropout(noise_shape=...) is not supported")
        self.rate = float(rate)
        self.noise_shape = noise_shape
        self.seed = seed
        if self._batch_input_shape is not None:
            self.build(self._batch_input_shape)

    def get_config(self):
        cfg = super().get_config()
        cfg.update({"rate": self.rate, "noise_shape": self.noise_shape, "seed": self.seed})
        return cfg


class Flatten(Layer):
    """Identity on the 2-D ``[batch, features]`` inputs this engine trains on."""

    def __init__(self, data_format=None, **kwargs):
        super().__init__(**kwargs)
        self.data_format = data_format
        if self._batch_input_shape is not None:
            self.build(self._batch_input_shape)

    def compute_output_shape(self, input_shape):
        n = 1
        for d in input_shape[1:]:
            n *= int(d)
        return (input_shape[0], n)

    def get_config(self):
        cfg = super().get_config()
        cfg["data_format"] = self.data_format or "channels_last"
        return cfg


LAYER_CLASSES = {c.__name__: c for c in (InputLayer, Dense, Activation, Dropout, Flatten)}


def deserialize(config: dict, custom_objects=None) -> Layer:
    cls_name = config["class_name"]
    if custom_objects and cls_name in custom_objects:
        cls = custom_objects[cls_name]
    elif cls_name in LAYER_CLASSES:
        cls = LAYER_CLASSES[cls_name]
    else:
        raise ValueError(f"Unknown layer: {cls_name}")
    cfg = dict(config["config"])
    if cls in (Dense, Activation):
        return cls.from_config(cfg, custom_objects)
    return cls.from_config(cfg)


def serialize(layer: Layer) -> dict:
    return {"class_name": type(layer).__name__, "config": layer.get_config()}
