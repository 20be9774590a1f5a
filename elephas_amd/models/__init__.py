"""Keras-compatible model API (Sequential / functional Model, Dense, Activation,
Dropout, losses, metrics, optimizers, HDF5 save/load) executed by the MI355X
native engine or the torch reference engine."""
from .layers import Activation, Dense, Dropout, Flatten, Input, InputLayer, Layer, clear_session
from .training import History, Model, Sequential, clone_model, model_from_config, model_from_json
from . import activations, backend, initializers, losses, metrics, optimizers


def load_model(filepath, custom_objects=None, compile=True):
    from ..io.keras_h5 import load_model as _lm
    return _lm(filepath, custom_objects=custom_objects, compile=compile)


def save_model(model, filepath, overwrite=True, include_optimizer=True):
    from ..io.keras_h5 import save_model as _sm
    _sm(model, filepath, overwrite=overwrite, include_optimizer=include_optimizer)


__all__ = ["Activation", "Dense", "Dropout", "Flatten", "Input", "InputLayer", "Layer", "History", "Model",
           "Sequential", "clone_model", "model_from_config", "model_from_json", "load_model", "save_model",
           "activations", "backend", "initializers", "losses", "metrics", "optimizers", "clear_session"]
