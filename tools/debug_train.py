import sys, os, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd import config
from elephas_amd.models import Sequential, Dense, Dropout
from elephas_amd.models.optimizers import SGD
from elephas_amd.ops.plan import build_plan
from elephas_amd.ops.native_engine import NativeTrainer
from elephas_amd.ops.torch_engine import TorchTrainer
from elephas_amd.models.datasets import synthetic_classification
x, y = synthetic_classification(4096, 784, 10, seed=5)
x = (x / 10).astype(np.float32); Y = np.eye(10, dtype=np.float32)[y]
for policy in ("float32", "mixed_bfloat16"):
    for drop in (0.0, 0.2):
        for shuffle in (False, True):
            config.set_policy(policy)
            np.random.seed(0)
            m = Sequential(); m.add(Dense(128, input_dim=784, activation='relu'))
            if drop: m.add(Dropout(drop))
            m.add(Dense(128, activation='relu'))
            if drop: m.add(Dropout(drop))
            m.add(Dense(10, activation='softmax'))
            m.compile(SGD(0.1), 'categorical_crossentropy', ['acc'])
            res = []
            for T in (NativeTrainer, TorchTrainer):
                t = T(m, build_plan(m), 1, 64, torch.device('cuda'))
                t.set_data([x], [Y], 0.1, shuffle=shuffle)
                h = t.fit(4)[0]
                res.append((round(h['loss'][0],3), round(h['loss'][-1],3), round(h['val_acc'][-1],3)))
            print(policy, drop, shuffle, 'native', res[0], 'torch', res[1], flush=True)
