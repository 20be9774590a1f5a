"""API reference generator (the reference's docs/autogen.py renders Keras-style
pages from docstrings). Walks the PAGES spec, renders each class / function
signature plus its docstring to Markdown under ``docs/sources`` and copies the
hand-written pages from ``docs/templates``.

    python docs/autogen.py [out_dir]
"""
from __future__ import annotations

import importlib
import inspect
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAGES = [
    ("models/spark-model.md", [
        "elephas_amd.spark_model.SparkModel", "elephas_amd.spark_model.SparkMLlibModel",
        "elephas_amd.spark_model.load_spark_model"]),
    ("models/spark-ml-model.md", [
        "elephas_amd.ml_model.ElephasEstimator", "elephas_amd.ml_model.ElephasTransformer",
        "elephas_amd.ml_model.load_ml_estimator", "elephas_amd.ml_model.load_ml_transformer"]),
    ("workers.md", ["elephas_amd.worker.SparkWorker", "elephas_amd.worker.AsynchronousSparkWorker"]),
    ("parameter/server.md", [
        "elephas_amd.parameter.server.BaseParameterServer", "elephas_amd.parameter.server.HttpServer",
        "elephas_amd.parameter.server.SocketServer", "elephas_amd.parameter.server.DeviceServer"]),
    ("parameter/client.md", [
        "elephas_amd.parameter.client.BaseParameterClient", "elephas_amd.parameter.client.HttpClient",
        "elephas_amd.parameter.client.SocketClient", "elephas_amd.parameter.client.DeviceClient"]),
    ("utils.md", [
        "elephas_amd.utils.rdd_utils", "elephas_amd.utils.functional_utils", "elephas_amd.utils.model_utils",
        "elephas_amd.utils.serialization", "elephas_amd.utils.sockets", "elephas_amd.utils.rwlock",
        "elephas_amd.utils.checkpoint"]),
    ("adapters.md", ["elephas_amd.ml.adapter", "elephas_amd.mllib.adapter"]),
    ("ml-params.md", ["elephas_amd.ml.params"]),
    ("profiling.md", ["elephas_amd.profiling"]),
    ("runtime.md", ["elephas_amd.ops.native_engine.NativeTrainer", "elephas_amd.ops.torch_engine.TorchTrainer",
                    "elephas_amd.ops.engine.make_trainer", "elephas_amd.parallel.dist"]),
]


def _resolve(path):
    try:
        return importlib.import_module(path)
    except ImportError:
        mod, _, name = path.rpartition(".")
        m = importlib.import_module(mod)
        return getattr(m, name, None)


def _sig(obj):
    try:
        return str(inspect.signature(obj))
    except (TypeError, ValueError):
        return "(...)"


def _doc(obj):
    return inspect.cleandoc(obj.__doc__) if obj.__doc__ else ""


def render(obj, name) -> str:
    out = []
    if inspect.ismodule(obj):
        out.append(f"## `{name}`\n\n{_doc(obj)}\n")
        for n, m in inspect.getmembers(obj):
            if n.startswith("_") or getattr(m, "__module__", None) != obj.__name__:
                continue
            if inspect.isfunction(m) or inspect.isclass(m):
                out.append(render(m, n))
        return "\n".join(out)
    if inspect.isclass(obj):
        out.append(f"### class `{name}{_sig(obj)}`\n\n{_doc(obj)}\n")
        for n, m in obj.__dict__.items():
            if n.startswith("_") and n != "__init__":
                continue
            if inspect.isfunction(m):
                out.append(f"#### `{name}.{n}{_sig(m)}`\n\n{_doc(m)}\n")
            elif isinstance(m, property):
                out.append(f"#### property `{name}.{n}`\n\n{_doc(m)}\n")
        return "\n".join(out)
    return f"### `{name}{_sig(obj)}`\n\n{_doc(obj)}\n"


def generate(out_dir: str) -> list:
    tpl = os.path.join(os.path.dirname(os.path.abspath(__file__)), "templates")
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    shutil.copytree(tpl, out_dir)
    written = []
    for page, names in PAGES:
        body = [f"# API: {os.path.splitext(os.path.basename(page))[0]}\n"]
        for n in names:
            obj = _resolve(n)
            if obj is None:
                raise ImportError(f"autogen: cannot resolve {n}")
            body.append(render(obj, n.rsplit(".", 1)[-1]))
        path = os.path.join(out_dir, "api", page)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write("\n".join(body))
        written.append(path)
    return written


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "sources")
    for p in generate(out):
        print(p)
