"""Phase timeline of the layer-pipeline kernel (csrc/kernels/deep_impl.h) from its in-kernel
s_memrealtime stamps (10 ns ticks): per step, the median (over the replica's workgroups)
of every phase's start / publication relative to the replica's median step start, and
the step period.

  python tools/deep_stamps.py [dims] [R] [B] [steps] [dropout] [sgd|adam]
  e.g. python tools/deep_stamps.py 93,512,512,512,9 8 128 8 0.5     (Otto, the default)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def names(L):
    n = {0: "start", 1: "dw0_done", 2: "fwd0_pub"}
    for l in range(1, L - 1):
        n[2 * l + 1] = f"fwd{l}_seen"
        n[2 * l + 2] = f"fwd{l}_pub"
    n.update({15: "fwd1_wt_staged", 16: "fwd1_ring_done", 17: "fwd1_ksred", 21: "tail_logits", 22: "tail_loss",
              23: "dwlast_done", 18: "bw_top_chunk0", 19: "bw_top_chunks", 24: "dw0_sync", 25: "xa_seen",
              26: "xb_seen", 27: "applied"})
    n[9] = "tail_seen"
    n[10] = "tail_pub"
    for l in range(L - 2, 0, -1):
        n[11 + 2 * (L - 2 - l)] = f"bw{l}_seen"
        n[12 + 2 * (L - 2 - l)] = f"bw{l}_pub"
    return n


def main():
    # dims as 93,512,512,512,9 or 93-512-512-512-9 (tools/gpu.py py: steps split on commas)
    dims = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "93,512,512,512,9").replace("-", ",").split(",")]
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    nst = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    drop = float(sys.argv[5]) if len(sys.argv) > 5 else 0.5
    opt = sys.argv[6] if len(sys.argv) > 6 else "sgd"
    os.environ.setdefault("ELEPHAS_AMD_DEEP", "2")
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, Dropout
    from elephas_amd.models.optimizers import SGD, Adam
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    m = Sequential()
    m.add(Dense(dims[1], activation="relu", input_dim=dims[0]))
    if drop:
        m.add(Dropout(drop))
    for d in dims[2:-1]:
        m.add(Dense(d, activation="relu"))
        if drop:
            m.add(Dropout(drop))
    m.add(Dense(dims[-1], activation="softmax"))
    m.compile(Adam(0.01) if opt == "adam" else SGD(0.01), "categorical_crossentropy", ["acc"])
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=1, persist=1)
    print("plan", t.plan_name())
    geo = t.exe.deep_geometry()
    if not geo:
        print("not on the layer pipeline:", t.plan_reason)
        return
    nw, grid, rt, ks, lds = geo[:5]
    print(f"nw {nw} grid {grid} RT {rt} KS {ks} LDS {lds} B")
    rng = np.random.default_rng(0)
    rows = B * 64
    xs = [rng.random((rows, dims[0]), dtype=np.float32) for _ in range(R)]
    ys = [np.eye(dims[-1], dtype=np.float32)[rng.integers(0, dims[-1], rows)] for _ in range(R)]
    t.set_data(xs, ys, 0.0)
    L = len(dims) - 1
    nm = names(L)
    st = torch.zeros(grid * 8 * 32, dtype=torch.int64, device="cuda")
    t.begin_epoch()
    t.run_steps(16)   # warm
    torch.cuda.synchronize()
    t.exe.set_stamps(st.data_ptr())
    for _ in range(3):
        st.zero_()
        torch.cuda.synchronize()
        t.exe.train_chunk(nst, t.s)
        torch.cuda.synchronize()
    t.exe.set_stamps(0)
    t.check()
    s = st.view(grid, 8, 32).cpu().numpy().astype(np.int64)
    rep = np.arange(grid) % R
    print("us relative to the replica's median step start (stamp 0); medians over workgroups")
    starts = []
    order = sorted(nm, key=lambda k: np.median(s[:, min(3, nst - 1), k][s[:, min(3, nst - 1), k] > 0]) if
                   (s[:, min(3, nst - 1), k] > 0).any() else 1e30)
    for i in range(min(8, nst)):
        b = np.zeros(grid)
        for rr in range(R):
            b[rep == rr] = np.median(s[rep == rr, i, 0])
        starts.append(np.median(b))
        vals = {}
        for k in order:
            n = nm[k]
            col = s[:, i, k]
            ok = col > 0
            if ok.any():
                vals[n] = np.median((col[ok] - b[ok]) / 100.0)
        print(f"step {i} " + " ".join(f"{k}={v:.2f}" for k, v in vals.items()))
    d = np.diff(starts) / 100.0
    print("step period (us):", np.round(d, 2), "median", np.round(np.median(d), 2) if len(d) else None)


if __name__ == "__main__":
    main()
