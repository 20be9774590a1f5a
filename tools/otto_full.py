"""The reference notebook's full Otto configuration (61,878 rows, 93-512-512-512-9,
Adam 0.01, 20 epochs, batch 128, validation_split 0.15, 1 worker) on the synthetic
Otto-shaped CSV, on whatever device is available; prints precision and wall time.
Reference value on the real Otto CSV: 0.764 (Spark_ML_Pipeline.ipynb:531)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
nb = json.load(open(os.path.join(ROOT, "examples", "Spark_ML_Pipeline.ipynb")))
os.chdir(tempfile.mkdtemp())
g, times = {}, []
for c in nb["cells"]:
    if c["cell_type"] != "code":
        continue
    t0 = time.perf_counter()
    exec(compile("".join(c["source"]).replace("os.path.abspath('..')", repr(ROOT)), "cell", "exec"), g)
    times.append(round(time.perf_counter() - t0, 2))
print(json.dumps({"precision": g["metrics"].precision(), "cell_seconds": times,
                  "device": str(__import__("elephas_amd").config.get_device())}))
