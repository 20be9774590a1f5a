import sys, os, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd import config
from elephas_amd.models import Sequential, Dense, Dropout
from elephas_amd.models.optimizers import SGD
from elephas_amd.ops.plan import build_plan
from elephas_amd.ops.native_engine import NativeTrainer
from elephas_amd.ops.torch_engine import TorchTrainer
from elephas_amd.models.datasets import synthetic_classification
config.set_policy("float32")
x, y = synthetic_classification(4096, 784, 10, seed=5)
x = (x / 10).astype(np.float32); Y = np.eye(10, dtype=np.float32)[y]
np.random.seed(0)
m = Sequential(); m.add(Dense(128, input_dim=784, activation='relu')); m.add(Dense(128, activation='relu')); m.add(Dense(10, activation='softmax'))
m.compile(SGD(0.1), 'categorical_crossentropy', ['acc'])
nat = NativeTrainer(m, build_plan(m), 1, 64, torch.device('cuda'))
ref = TorchTrainer(m, build_plan(m), 1, 64, torch.device('cuda'))
for t in (nat, ref): t.set_data([x], [Y], 0.1, shuffle=False)
print("ntrain", nat.ntrain_h, nat.vcount_h, "steps/epoch", nat.steps_per_epoch())
nat.begin_epoch()
for k in range(1, 60):
    nat.run_steps(1, use_graph=False)
    i0 = (k - 1) * 64
    ref.train_batch(0, ref.xs[0][i0:i0 + 64], ref.ys[0][i0:i0 + 64])
    if k in (1, 2, 3, 5, 10, 20, 40, 57, 58, 59):
        wn, wr = nat.get_weights_flat()[0], ref.get_weights_flat()[0]
        print(k, "ctr", nat.ctr.cpu().numpy().tolist(), "maxdiff", float(np.abs(wn - wr).max()), "acc", nat.acc.cpu().numpy()[0][:3].tolist(), flush=True)
print("eval native", nat.evaluate(x[:500], Y[:500]), "ref", ref.evaluate(x[:500], Y[:500]))
print("val sums", nat._val_sums()[0][:3])
