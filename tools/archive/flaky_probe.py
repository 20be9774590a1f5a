"""Repeat the fp32 one-step native-vs-torch comparison many times in one process
(fresh engines each time) and print the relative error per trial and per layer,
to catch nondeterministic (timing- or placement-dependent) divergence."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_native_gpu import _mlp, _data, _engines  # noqa: E402
from elephas_amd.models import optimizers as O  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 20
policy = sys.argv[2] if len(sys.argv) > 2 else "float32"
bad = 0
for t in range(trials):
    model = _mlp(784, [128, 128], 10)
    model.compile(O.SGD(0.1), "categorical_crossentropy", ["acc"])
    x, y = _data(64, 784, 10)
    nat, ref = _engines(model, 64, policy)
    for e in (nat, ref):
        e.set_data([x], [y], 0.0, shuffle=False)
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    errs = []
    for step in range(3):
        nat.fit(2 if step == 0 else 1)  # the unit test's fit(2) first
        ref.fit(2 if step == 0 else 1)
        wn, wr = nat.get_weights_flat()[0], ref.get_weights_flat()[0]
        errs.append(float(np.abs(wn - wr).max() / max(np.abs(wr - w0).max(), 1e-12)))
    sizes = [w.size for w in model.get_weights()]
    offs = np.cumsum([0] + sizes)
    per = [float(np.abs(wn[a:b] - wr[a:b]).max()) for a, b in zip(offs[:-1], offs[1:])]
    flag = errs[-1] > 1e-3
    bad += flag
    print(f"trial {t} errs {['%.2e' % e for e in errs]} per-tensor {['%.1e' % p for p in per]}{' BAD' if flag else ''}",
          flush=True)
print(f"bad {bad}/{trials}")
