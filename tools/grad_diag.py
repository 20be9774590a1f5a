"""Which gradient elements of the multi-launch plans deviate on one batch (the sync test's
shard 2, R = 1): native G (forward_backward) vs torch autograd, per layer -- the worst
elements' (row, col) positions and the pattern over row / column tiles."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_deep_gpu import _mlp, _shards
    from elephas_amd import config
    from elephas_amd.models import initializers, optimizers as O
    from elephas_amd.ops.plan import build_plan, unflatten_weights
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    initializers.set_seed(12)
    in_dim, hidden, out, B = 93, (256, 256, 128), 9, 128
    model = _mlp(in_dim, list(hidden), out)
    model.compile(O.SGD(0.05), "categorical_crossentropy", ["acc"])
    like = model.get_weights()
    xs, ys = _shards([B * 5] * 4, in_dim, out, seed=13)
    shard = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    x, y = xs[shard][:B], ys[shard][:B]
    ws = [torch.tensor(w, device="cuda", requires_grad=True) for w in like]
    h = torch.tensor(x, device="cuda")
    zs = []
    for i in range(0, len(ws), 2):
        z = h @ ws[i] + ws[i + 1]
        zs.append(z)
        h = torch.relu(z) if i + 2 < len(ws) else z
    loss = torch.nn.functional.cross_entropy(h, torch.tensor(y, device="cuda").argmax(1))
    gt = torch.autograd.grad(loss, ws)
    for i, z in enumerate(zs[:-1]):
        zz = z.detach().cpu().numpy()
        print(f"Z_{i}: exact zeros {int((zz == 0).sum())}, |z| < 1e-6: {int((np.abs(zz) < 1e-6).sum())}, "
              f"rows with no positive unit {int(((zz > 0).sum(1) == 0).sum())}", flush=True)
    for env in ("-1", "0"):
        os.environ["ELEPHAS_AMD_ROWCHAIN"] = env
        t = NativeTrainer(model, build_plan(model), 1, B, torch.device("cuda"), seed=5, persist=0)
        t.set_data([xs[shard]], [ys[shard]], 0.0, shuffle=False)
        t.begin_epoch()
        t._ensure_images()
        t.exe.forward_backward(t.s)
        torch.cuda.synchronize()
        g = t.G[0].detach().cpu().numpy()
        for li, (gn, gr) in enumerate(zip(unflatten_weights(g, like), gt)):
            gr = gr.detach().cpu().numpy()
            d = np.abs(gn - gr)
            rel = d.max() / (np.abs(gr).max() + 1e-30)
            msg = f"plan {t.plan_name()[:22]!r} param {li} shape {gr.shape} max rel err {rel:.2e}"
            if rel > 1e-4 and gr.ndim == 2:
                bad = d > 1e-3 * np.abs(gr).max()
                rows, cols = np.nonzero(bad)
                msg += (f"; bad {bad.sum()} elements, rows {np.unique(rows)[:20]}..., cols tiles16 "
                        f"{np.unique(cols // 16)}, row tiles16 {np.unique(rows // 16)}")
            elif rel > 1e-4:
                msg += f"; bad idx {np.nonzero(d > 1e-3 * np.abs(gr).max())[0][:20]}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()
