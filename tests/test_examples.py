"""The ported reference examples (examples/*.py, reference examples/) run end to
end on the CPU engine with trimmed synthetic data."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


@pytest.mark.parametrize("script,expect", [
    ("mnist_mlp_spark_synchronous.py", "Test accuracy"),
    ("mnist_mlp_spark_asynchronous.py", "Test accuracy"),
    ("mllib_mlp.py", "Test accuracy"),
    ("ml_mlp_regression.py", ""),
    ("ml_pipeline_otto.py", "precision"),
])
def test_example_runs(tmp_path, script, expect):
    env = dict(os.environ, PYTHONPATH=ROOT, EXAMPLE_ROWS="800", EXAMPLE_EPOCHS="1", OTTO_ROWS="600",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    if script == "ml_pipeline_otto.py":   # writes its synthetic CSV next to a copy of the script
        import shutil
        shutil.copy(os.path.join(EX, script), tmp_path / script)
        cwd, path = str(tmp_path), str(tmp_path / script)
    else:
        cwd, path = EX, os.path.join(EX, script)
    r = subprocess.run([sys.executable, path], cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert expect in r.stdout


def test_notebook_cells_run(tmp_path, monkeypatch):
    """examples/Spark_ML_Pipeline.ipynb (reference notebook port): execute its code
    cells in order with a smaller synthetic CSV and 2 epochs."""
    import json
    nb = json.load(open(os.path.join(EX, "Spark_ML_Pipeline.ipynb")))
    monkeypatch.chdir(tmp_path)
    g = {}
    for c in nb["cells"]:
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"]).replace("os.path.abspath('..')", repr(ROOT))
        src = src.replace("61878", "600").replace("set_epochs(20)", "set_epochs(1)")
        exec(compile(src, "cell", "exec"), g)
    assert 0.0 <= g["metrics"].precision() <= 1.0


def test_notebook_otto_pipeline_learns(tmp_path, monkeypatch):
    """Learnability bar for the Otto pipeline (the reference's only quality number is
    train precision 0.764 on the real Otto CSV, Spark_ML_Pipeline.ipynb:531; that CSV is
    not available offline, so parity with 0.764 is unpinned).  The notebook's synthetic
    Otto-shaped data has overlapping classes (shared Poisson rates, +-25 % per class);
    6000 rows x 4 epochs of the notebook's model and Adam config must reach precision
    0.75 (measured 0.83 on the CPU engine; untrained: ~0.11)."""
    import json
    nb = json.load(open(os.path.join(EX, "Spark_ML_Pipeline.ipynb")))
    monkeypatch.chdir(tmp_path)
    g = {}
    for c in nb["cells"]:
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"]).replace("os.path.abspath('..')", repr(ROOT))
        src = src.replace("61878", "6000").replace("set_epochs(20)", "set_epochs(4)")
        exec(compile(src, "cell", "exec"), g)
    assert g["metrics"].precision() >= 0.75
