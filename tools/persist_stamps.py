"""Phase timeline of the persistent step kernel (csrc/kernels/persist.hip) from its
in-kernel s_memrealtime stamps (10 ns ticks): per step, every phase of the chain and
layer-0 workgroups relative to the moment the chain workgroups saw the step's partials.

  python tools/persist_stamps.py [R] [B] [steps]
"""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    nst = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, Dropout
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    m = Sequential()
    m.add(Dense(128, activation="relu", input_dim=784))
    m.add(Dropout(0.2))
    m.add(Dense(128, activation="relu"))
    m.add(Dropout(0.2))
    m.add(Dense(10, activation="softmax"))
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=1, persist=1)
    rng = np.random.default_rng(0)
    xs = [rng.random((7500, 784), dtype=np.float32) for _ in range(R)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(R)]
    t.set_data(xs, ys, 0.1)
    nk0, nc0, kc0, cw, nch, wgs, grid = t.exe.persist_geometry()
    print("geometry", dict(nk0=nk0, nc0=nc0, kc0=kc0, cw=cw, nch=nch, wgs=wgs, grid=grid))
    st = torch.zeros(grid * 8 * 16, dtype=torch.int64, device="cuda")
    t.begin_epoch()
    t.run_steps(32, use_graph=False)   # warm
    torch.cuda.synchronize()
    t.exe.set_stamps(st.data_ptr())
    t.exe.train_step(t.s) if nst == 1 else None
    for _ in range(3):
        st.zero_()
        torch.cuda.synchronize()
        # one launch of nst steps (eager chunk through a fresh capture-less path)
        g = t.exe.capture(nst, 0, t.s)
        t.exe.replay(g, t.s)
        torch.cuda.synchronize()
    t.check()
    s = st.view(grid, 8, 16).cpu().numpy().astype(np.int64)
    nl0 = nk0 * nc0
    q = np.arange(grid) // R
    chain = q >= nl0
    l0 = ~chain
    base_all = s[chain, :, 1]   # chain: partials seen
    print("ticks of 10 ns; per step (median over workgroups) relative to the chain's partial-wait end")
    names_c = ["part_wait0", "part_seen", "phase0", "fwd1", "fwd2+loss", "dx2+dx1", "bwd_pub", "bwd_seen",
               "stage_ld", "dw_upd", "w_pub", "w_seen", "w_loaded"]
    names_l = ["start", "part_pub", "bwd_wait0", "bwd_seen", "dz_ld", "dw_upd", "fwd_done"]
    for i in range(min(8, nst)):
        b0 = np.median(base_all[:, i])
        if b0 == 0:
            continue
        c = {n: (np.median(s[chain, i, k]) - b0) / 100.0 for k, n in enumerate(names_c) if (s[chain, i, k] > 0).all()}
        l = {n: (np.median(s[l0, i, k]) - b0) / 100.0 for k, n in enumerate(names_l) if (s[l0, i, k] > 0).all()}
        print(f"step {i}: chain " + " ".join(f"{k}={v:.2f}" for k, v in c.items()))
        print(f"        l0    " + " ".join(f"{k}={v:.2f}" for k, v in l.items()))
    steps = [np.median(base_all[:, i]) for i in range(min(8, nst))]
    d = np.diff([x for x in steps if x > 0]) / 100.0
    print("step period (us):", np.round(d, 2))


if __name__ == "__main__":
    main()
