"""Keras-compatible model API on the torch reference engine (CPU)."""
import json

import numpy as np
import pytest
import torch

from elephas_amd.models import (Activation, Dense, Dropout, Input, Model, Sequential, load_model,
                                model_from_json)
from elephas_amd.models import losses as L
from elephas_amd.models import metrics as M
from elephas_amd.models import optimizers as O


def test_sequential_json_roundtrip(classification_model):
    js = classification_model.to_json()
    cfg = json.loads(js)
    assert cfg["class_name"] == "Sequential"
    assert cfg["config"]["layers"][0]["class_name"] == "InputLayer"
    assert cfg["config"]["layers"][0]["config"]["batch_input_shape"] == [None, 784]
    assert model_from_json(js).to_json() == js


def test_functional_json_roundtrip(classification_model_functional):
    js = classification_model_functional.to_json()
    m = model_from_json(js)
    assert m.to_json() == js
    assert [w.shape for w in m.get_weights()] == [(784, 128), (128,), (128, 128), (128,), (128, 10), (10,)]


def test_weights_order_and_count(classification_model):
    ws = classification_model.get_weights()
    assert [w.shape for w in ws] == [(784, 128), (128,), (128, 128), (128,), (128, 10), (10,)]
    assert classification_model.count_params() == 118282
    b = ws[1]
    assert np.all(b == 0)   # zeros bias init
    lim = np.sqrt(6 / (784 + 128))
    assert np.abs(ws[0]).max() <= lim + 1e-6   # glorot uniform


def test_compile_required_and_attributes(regression_model):
    assert not hasattr(regression_model, "loss")
    with pytest.raises(RuntimeError):
        regression_model.fit(np.zeros((4, 13)), np.zeros(4))
    regression_model.compile("sgd", "mse", ["mae"])
    assert regression_model.loss == "mse"
    assert regression_model.compiled_metrics._metrics == ["mae"]
    assert regression_model.metrics_names == ["loss", "mae"]


def test_fit_history_and_validation_split(classification_model, mnist_data):
    x, y, xt, yt = mnist_data
    classification_model.compile(O.SGD(lr=0.1), "categorical_crossentropy", ["acc"])
    h = classification_model.fit(x[:640], y[:640], batch_size=64, epochs=2, verbose=0, validation_split=0.1)
    assert set(h.history) == {"loss", "acc", "val_loss", "val_acc"}
    assert len(h.history["loss"]) == 2 and h.epoch == [0, 1]
    res = classification_model.evaluate(xt, yt, verbose=0)
    assert isinstance(res, list) and len(res) == 2
    p = classification_model.predict(xt[:5])
    assert p.shape == (5, 10) and np.allclose(p.sum(1), 1, atol=1e-5)


def test_evaluate_scalar_without_metrics(regression_model, boston_housing_dataset):
    x, y, xt, yt = boston_housing_dataset
    regression_model.compile(O.SGD(learning_rate=1e-7), "mse")
    regression_model.fit(x, y, epochs=1, batch_size=64, verbose=0)
    assert isinstance(regression_model.evaluate(xt, yt), float)


def test_train_on_batch_matches_manual_sgd():
    m = Sequential([Dense(3, input_dim=4, activation="linear")])
    m.compile(O.SGD(0.5), "mse")
    w0, b0 = [w.copy() for w in m.get_weights()]
    x = np.random.default_rng(0).normal(size=(8, 4)).astype(np.float32)
    y = np.random.default_rng(1).normal(size=(8, 3)).astype(np.float32)
    loss = m.train_on_batch(x, y)
    pred = x @ w0 + b0
    g = 2 * (pred - y) / (8 * 3)
    assert np.isclose(loss, np.mean((pred - y) ** 2), rtol=1e-5)
    assert np.allclose(m.get_weights()[0], w0 - 0.5 * x.T @ g, atol=1e-5)
    assert np.allclose(m.get_weights()[1], b0 - 0.5 * g.sum(0), atol=1e-5)


@pytest.mark.parametrize("name", list(L.FUNCTIONS))
def test_losses_finite_and_differentiable(name):
    rng = np.random.default_rng(0)
    if name == "sparse_categorical_crossentropy":
        yt = torch.tensor(rng.integers(0, 5, (6, 1)).astype(np.float32))
    else:
        yt = torch.tensor(rng.random((6, 5)).astype(np.float32))
    z = torch.tensor(rng.normal(size=(6, 5)).astype(np.float32), requires_grad=True)
    p = torch.softmax(z, -1)
    v = L.FUNCTIONS[name](yt, p)
    assert v.shape == (6,) and torch.isfinite(v).all()
    v.sum().backward()
    assert torch.isfinite(z.grad).all()


def test_cce_logits_path_equals_clipped_path():
    z = torch.randn(4, 10)
    y = torch.nn.functional.one_hot(torch.arange(4), 10).float()
    a = L.categorical_crossentropy(y, torch.softmax(z, -1), logits=z)
    b = L.categorical_crossentropy(y, torch.softmax(z, -1))
    assert torch.allclose(a, b, atol=1e-5)


def test_accuracy_resolution():
    cce = L.get("categorical_crossentropy")
    assert M.MetricSpec("acc", 10, cce).native == M.MET_ACC_CAT
    assert M.MetricSpec("accuracy", 1, L.get("binary_crossentropy")).native == M.MET_ACC_BIN
    assert M.MetricSpec("acc", 10, L.get("sparse_categorical_crossentropy")).native == M.MET_ACC_SPARSE
    assert M.MetricSpec("mae", 1, cce).name == "mae"


def test_optimizer_serialization_roundtrip():
    sgd = O.SGD(learning_rate=0.01, decay=1e-6, momentum=0.9, nesterov=True)
    conf = O.serialize(sgd)
    assert conf["class_name"] == "SGD"
    assert conf["config"]["momentum"] == 0.9 and conf["config"]["decay"] == 1e-6
    back = O.deserialize(conf)
    assert O.serialize(back) == conf
    assert isinstance(O.get("adam"), O.Adam) and O.get("rmsprop").learning_rate == 0.001
    assert O.SGD(lr=0.1).learning_rate == 0.1   # legacy lr=


def _numpy_adam(w, gs, lr=0.01, b1=0.9, b2=0.999, eps=1e-7):
    m = np.zeros_like(w)
    v = np.zeros_like(w)
    for t, g in enumerate(gs, 1):
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        w = w - lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t) * m / (np.sqrt(v) + eps)
    return w


def test_adam_rule_matches_keras_formula():
    opt = O.Adam(0.01)
    w = torch.ones(5)
    st = opt.init_state([w])
    gs = [np.random.default_rng(i).normal(size=5).astype(np.float32) for i in range(3)]
    for i, g in enumerate(gs):
        opt.apply_torch([w], [torch.tensor(g)], st[0:1], i)
    assert np.allclose(w.numpy(), _numpy_adam(np.ones(5, np.float32), gs), atol=1e-6)


# Independent numpy transcriptions of the Keras 2.10 optimizer_v2 update rules
# (keras/optimizers/optimizer_v2/*.py and the tf.raw_ops.ResourceApply* kernels they
# call); lr_t = lr / (1 + decay * iterations) with iterations counted from 0.
def _keras_rule(name, hp):
    def sgd(w, g, st, it):
        lr = hp["lr"] / (1 + hp.get("decay", 0) * it)
        mom = hp.get("momentum", 0)
        if mom == 0:
            return w - lr * g
        st["m"] = mom * st.get("m", 0) - lr * g
        return w + mom * st["m"] - lr * g if hp.get("nesterov") else w + st["m"]

    def rmsprop(w, g, st, it):
        lr = hp["lr"] / (1 + hp.get("decay", 0) * it)
        rho, eps, mom = hp.get("rho", 0.9), hp.get("eps", 1e-7), hp.get("momentum", 0)
        st["ms"] = st.get("ms", 0) + (g * g - st.get("ms", 0)) * (1 - rho)
        denom = st["ms"]
        if hp.get("centered"):
            st["mg"] = st.get("mg", 0) + (g - st.get("mg", 0)) * (1 - rho)
            denom = denom - st["mg"] ** 2
        if mom:                                   # ResourceApplyRMSProp: eps inside sqrt
            st["mom"] = mom * st.get("mom", 0) + lr * g / np.sqrt(denom + eps)
            return w - st["mom"]
        return w - lr * g / (np.sqrt(denom) + eps)

    def adagrad(w, g, st, it):
        lr = hp["lr"] / (1 + hp.get("decay", 0) * it)
        st["acc"] = st.get("acc", hp.get("init", 0.1)) + g * g
        return w - lr * g / (np.sqrt(st["acc"]) + hp.get("eps", 1e-7))

    def adamax(w, g, st, it):
        lr = hp["lr"] / (1 + hp.get("decay", 0) * it)
        b1, b2, eps = 0.9, 0.999, 1e-7
        st["m"] = b1 * st.get("m", 0) + (1 - b1) * g
        st["u"] = np.maximum(b2 * st.get("u", 0), np.abs(g))
        return w - lr / (1 - b1 ** (it + 1)) * st["m"] / (st["u"] + eps)
    return {"sgd": sgd, "rmsprop": rmsprop, "adagrad": adagrad, "adamax": adamax}[name]


@pytest.mark.parametrize("name,opt,hp", [
    ("sgd", lambda: O.SGD(0.05), {"lr": 0.05}),
    ("sgd", lambda: O.SGD(0.05, momentum=0.9), {"lr": 0.05, "momentum": 0.9}),
    ("sgd", lambda: O.SGD(0.01, decay=1e-2, momentum=0.9, nesterov=True),
     {"lr": 0.01, "decay": 1e-2, "momentum": 0.9, "nesterov": True}),
    ("rmsprop", lambda: O.RMSprop(0.01), {"lr": 0.01}),
    ("rmsprop", lambda: O.RMSprop(0.01, momentum=0.5, decay=0.1), {"lr": 0.01, "momentum": 0.5, "decay": 0.1}),
    ("rmsprop", lambda: O.RMSprop(0.01, centered=True), {"lr": 0.01, "centered": True}),
    ("rmsprop", lambda: O.RMSprop(0.01, centered=True, momentum=0.3),
     {"lr": 0.01, "centered": True, "momentum": 0.3}),
    ("adagrad", lambda: O.Adagrad(0.1), {"lr": 0.1}),
    ("adagrad", lambda: O.Adagrad(0.1, initial_accumulator_value=0.5, decay=0.05),
     {"lr": 0.1, "init": 0.5, "decay": 0.05}),
    ("adamax", lambda: O.Adamax(0.02), {"lr": 0.02}),
])
def test_optimizer_rules_match_keras_formulas(name, opt, hp):
    """Every optimizer of the engines (the torch rule here; the native kernels are
    checked against the torch engine on the GPU) against the Keras formulas, 4 steps."""
    o = opt()
    w = torch.linspace(-1, 1, 7)
    st = o.init_state([w])
    ref_w, ref_st = w.numpy().astype(np.float64).copy(), {}
    rule = _keras_rule(name, hp)
    for it in range(4):
        g = np.random.default_rng(40 + it).normal(size=7).astype(np.float32)
        o.apply_torch([w], [torch.tensor(g)], st[0:1], it)
        ref_w = rule(ref_w, g.astype(np.float64), ref_st, it)
    np.testing.assert_allclose(w.numpy(), ref_w, rtol=1e-5, atol=1e-6)


def test_save_load_roundtrip(tmp_cwd, classification_model):
    classification_model.compile(O.RMSprop(), "categorical_crossentropy", ["acc"])
    classification_model.save("model.h5")
    m = load_model("model.h5")
    assert m.to_json() == classification_model.to_json()
    assert all(np.array_equal(a, b) for a, b in zip(m.get_weights(), classification_model.get_weights()))
    assert isinstance(m.optimizer, O.RMSprop) and m.loss == "categorical_crossentropy"


def test_custom_activation_runs_on_torch_engine():
    from elephas_amd.models import backend as K

    def custom_activation(x):
        return K.sigmoid(x) + 1
    m = Sequential()
    m.add(Dense(1, input_dim=1, activation=custom_activation))
    m.add(Dense(1, activation="sigmoid"))
    m.compile(O.SGD(learning_rate=0.1), "binary_crossentropy", ["acc"])
    x = np.random.rand(100)
    y = np.zeros(100)
    y[:50] = 1
    m.fit(x, y, epochs=1, batch_size=16, verbose=0)
    assert m.predict(np.random.rand(10)).shape == (10, 1)
    js = m.to_json()
    assert "custom_activation" in js
    with pytest.raises(ValueError):
        model_from_json(js)
    assert model_from_json(js, {"custom_activation": custom_activation}).to_json() == js
