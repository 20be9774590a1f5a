"""Diagnose the split-K wide last layer: predictions (forward only) and one training
step of the native engine vs the fp32 torch engine, split on and off."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_native_gpu as T  # noqa: E402
from elephas_amd.models import initializers  # noqa: E402

initializers.set_seed(5)
model = T._mlp(64, [2048], 300)
model.compile("sgd", "categorical_crossentropy", ["acc"])
x, y = T._data(600, 64, 300, seed=6)
nat, ref = T._engines(model, 256, "float32")
pn, pr = nat.predict(x[:300]), ref.predict(x[:300])
print("predict max abs diff", float(np.abs(pn - pr).max()), "max p", float(pr.max()))
for steps in (1, 2, 3):
    nat, ref = T._engines(model, 256, "float32")
    w0 = nat.get_weights_flat()[0].copy()
    for t in (nat, ref):
        t.set_data([x], [y], 0.0, shuffle=False)
        t.begin_epoch() if hasattr(t, "begin_epoch") else None
    nat.run_steps(steps, use_graph=False)
    ref.train_steps(steps)
    wn, wr = nat.get_weights_flat()[0], ref.get_weights_flat()[0]
    d = np.abs(wn - wr)
    print(f"steps {steps}: max diff {d.max():.3e} at {int(d.argmax())} of {d.size}; max update {np.abs(wr - w0).max():.3e}")

# error pattern of the forward: which rows / columns of the logits are wrong
initializers.set_seed(5)
model = T._mlp(64, [2048], 300, out_act="linear")
model.compile("sgd", "mse")
nat, ref = T._engines(model, 256, "float32")
pn, pr = nat.predict(x[:300]), ref.predict(x[:300])
e = np.abs(pn - pr)
cols = e.max(0)
rows = e.max(1)
print("linear logits: max err", float(e.max()), "typical |z|", float(np.abs(pr).mean()))
print("bad columns:", np.nonzero(cols > 1e-4)[0][:40].tolist(), "count", int((cols > 1e-4).sum()))
print("bad rows:", np.nonzero(rows > 1e-4)[0][:40].tolist(), "count", int((rows > 1e-4).sum()))
ratio = (pn / np.where(np.abs(pr) > 1e-6, pr, np.nan))
print("median ratio native/ref", float(np.nanmedian(ratio)))
