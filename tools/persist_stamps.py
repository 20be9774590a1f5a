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
    st = torch.zeros(grid * 8 * 32, dtype=torch.int64, device="cuda")
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
    s = st.view(grid, 8, 32).cpu().numpy().astype(np.int64)
    nl0 = nk0 * nc0
    q = np.arange(grid) // R
    chain = q >= nl0
    l0 = ~chain
    base_all = s[chain, :, 1]   # chain: partials seen
    print("ticks of 10 ns; per step (median over workgroups) relative to the chain's partial-wait end")
    names_c = {0: "part_wait0", 1: "part_seen", 13: "p0_loads", 14: "p0_act", 15: "p0_st", 2: "phase0",
               16: "fwd1_mm", 17: "fwd1_epi", 3: "fwd1", 18: "fwd2", 19: "logits", 20: "loss", 4: "dz2",
               21: "dx2", 22: "dz1_pub", 23: "dx1_mm", 5: "dx1", 6: "bwd_pub", 7: "bwd_seen",
               8: "stage_ld", 24: "dw_mm", 25: "colsum", 26: "opt", 9: "upd", 10: "w_pub"}
    names_l = {0: "start", 1: "part_pub", 2: "bwd_wait0", 3: "bwd_seen", 4: "dz_ld", 7: "dw_mm", 8: "colsum",
               9: "opt", 5: "dw_upd", 10: "fwd_mm", 6: "fwd_done"}
    for i in range(min(8, nst)):
        b0 = np.median(base_all[:, i])
        if b0 == 0:
            continue
        c = {n: (np.median(s[chain, i, k]) - b0) / 100.0 for k, n in names_c.items() if (s[chain, i, k] > 0).all()}
        l = {n: (np.median(s[l0, i, k]) - b0) / 100.0 for k, n in names_l.items() if (s[l0, i, k] > 0).all()}
        print(f"step {i}: chain " + " ".join(f"{k}={v:.2f}" for k, v in c.items()))
        print(f"        l0    " + " ".join(f"{k}={v:.2f}" for k, v in l.items()))
    cyc = (s[chain, 1:7, 29] - s[chain, 1:7, 28]).astype(np.float64)
    rt = (s[chain, 1:7, 10] - s[chain, 1:7, 13]).astype(np.float64) / 100.0
    print("chain shader clock (MHz, median):", np.median(cyc / np.maximum(rt, 1e-9)))
    steps = [np.median(base_all[:, i]) for i in range(min(8, nst))]
    d = np.diff([x for x in steps if x > 0]) / 100.0
    print("step period (us):", np.round(d, 2))


if __name__ == "__main__":
    main()
