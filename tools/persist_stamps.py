"""Phase timeline of the persistent step kernel (csrc/kernels/persist.hip) from its
in-kernel s_memrealtime stamps (10 ns ticks): per step, the median stamp of every
phase of every role relative to the chain workgroups' publication of the previous
step's dZ_0 rows (V2: the step's true start; V1: the partials seen), and the step period.

  python tools/persist_stamps.py [R] [B] [steps] [v2: 1|0|-1] [policy] [sync]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = {
    "chain": {0: "part_wait0", 1: "part_dz0_seen", 11: "gram_ld", 12: "w_seen", 13: "p0_sums",
              27: "correction", 14: "p0_act", 15: "p0_st", 2: "phase0", 16: "fwd1_mm", 17: "fwd1_epi",
              3: "fwd1", 18: "fwd2", 19: "logits", 20: "loss", 4: "dz2", 21: "dx2", 22: "dz1_pub",
              23: "dx1_mm", 5: "dx1", 6: "bwd_pub", 7: "bwd_seen", 8: "stage_ld", 24: "dw_mm", 26: "opt",
              9: "upd", 10: "w_pub"},
    "l0": {0: "start", 1: "part_pub", 9: "x_next", 10: "gram_next", 2: "bwd_wait0", 3: "bwd_seen", 4: "dz_ld",
           7: "dw_mm", 8: "colsum", 5: "dw_upd", 6: "next_pub"},
    "dw": {0: "a0_wait0", 1: "a0_seen", 2: "d2_seen", 3: "staged", 4: "dz1", 5: "dw_mm", 6: "w_pub", 7: "gram"},
}


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    nst = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    if len(sys.argv) > 4 and sys.argv[4] != "-1":
        os.environ["ELEPHAS_AMD_PERSIST_V2"] = sys.argv[4]
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, Dropout
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy(sys.argv[5] if len(sys.argv) > 5 else "float32")
    m = Sequential()
    m.add(Dense(128, activation="relu", input_dim=784))
    m.add(Dropout(0.2))
    m.add(Dense(128, activation="relu"))
    m.add(Dropout(0.2))
    m.add(Dense(10, activation="softmax"))
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    sync = len(sys.argv) > 6 and sys.argv[6] == "sync"
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=1, persist=1, sync=sync)
    rng = np.random.default_rng(0)
    xs = [rng.random((7500, 784), dtype=np.float32) for _ in range(R)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(R)]
    t.set_data(xs, ys, 0.1)
    nk0, nc0, kc0, cw, nch, wgs, grid = t.exe.persist_geometry()
    var, nd, sync = t.exe.persist_variant()[:3]
    print("plan", t.plan_name())
    st = torch.zeros(grid * 8 * 32, dtype=torch.int64, device="cuda")
    t.begin_epoch()
    t.run_steps(32)   # warm
    torch.cuda.synchronize()
    t.exe.set_stamps(st.data_ptr())
    for _ in range(3):
        st.zero_()
        torch.cuda.synchronize()
        t.exe.train_chunk(nst, t.s)
        torch.cuda.synchronize()
    t.check()
    s = st.view(grid, 8, 32).cpu().numpy().astype(np.int64)
    nl0 = nk0 * nc0
    bidx = np.arange(grid)
    if t.exe.persist_variant()[3] == 2:   # exchange-local instance: the 8 copies of workgroup q on one XCD
        q = (bidx & 7) + 8 * (bidx >> 6)
        rep = (bidx >> 3) & 7
    else:
        q = bidx // R
        rep = bidx % R
    roles = {"l0": q < nl0, "chain": (q >= nl0) & (q < nl0 + nch), "dw": q >= nl0 + nch}
    chain = roles["chain"]
    ref_k = 6   # chain: dZ_0 rows published (end of a step)
    print("ticks of 10 ns -> us; per step, medians relative to the same replica's chains' dZ_0 "
          "publication of the previous step (replicas run unsynchronised)")

    def base(i):   # per block: its replica's median chain dZ_0 publication of step i - 1
        b = np.zeros(grid)
        for rr in range(R):
            b[rep == rr] = np.median(s[chain & (rep == rr), i - 1, ref_k])
        return b

    for i in range(1, min(8, nst)):
        b0 = base(i)
        if (b0 == 0).any():
            continue
        for role, mask in roles.items():
            if not mask.any():
                continue
            vals = {n: np.median((s[mask, i, k] - b0[mask]) / 100.0) for k, n in NAMES[role].items()
                    if (s[mask, i, k] > 0).all()}
            print(f"step {i} {role:5s} " + " ".join(f"{k}={v:.2f}" for k, v in vals.items()))
    # spread of the hand-offs within a replica: the last chain's dZ_0 publication, the
    # last PART publication (layer-0 iteration i - 2), each chain's wait end
    for i in range(2, min(8, nst)):
        b0 = base(i)
        if (b0 == 0).any():
            continue
        cl, pl, sl, jl = [], [], [], []
        for rr in range(R):
            m = rep == rr
            cl.append((s[chain & m, i - 1, ref_k].max() - b0[m][0]) / 100.0)
            pl.append((s[roles["l0"] & m, i - 2, 6].max() - b0[m][0]) / 100.0)
            sl.append((s[chain & m, i, 1].max() - b0[m][0]) / 100.0)
            jl.append([(s[chain & m & (q == nl0 + j), i - 1, ref_k][0] - b0[m][0]) / 100.0 for j in range(nch)])
        print(f"step {i} last dz0_pub(i-1) {np.round(np.median(cl), 2)}  last part_pub {np.round(np.median(pl), 2)}"
              f"  last seen {np.round(np.median(sl), 2)}  per chain j dz0_pub {np.round(np.median(jl, axis=0), 2)}")
    if sync:
        # the replica exchange of every owning workgroup q (absolute times, all replicas):
        # skew = last replica's arrival - this replica's, latency = this replica's exit - last arrival
        for role, (ka, kb) in (("l0", (7, 8)), ("chain", (24, 26))):
            sk, lat = [], []
            for i in range(1, min(8, nst)):
                for qq in np.unique(q[roles[role]]):
                    m = q == qq
                    a_, b_ = s[m, i, ka], s[m, i, kb]
                    if (a_ == 0).any() or (b_ == 0).any():
                        continue
                    sk.extend((a_.max() - a_) / 100.0)
                    lat.extend((b_ - a_.max()) / 100.0)
            if sk:
                print(f"exchange {role}: wait for the last replica median {np.median(sk):.2f} us (max {np.max(sk):.2f}); "
                      f"after the last arrival median {np.median(lat):.2f} us (min {np.min(lat):.2f})")
    # the launch's fill: step 0 relative to the earliest layer-0 start stamp of the replica
    f = {}
    for rr in range(R):
        m = rep == rr
        t0 = s[roles["l0"] & m, 0, 0].min()
        f.setdefault("l0 part_pub(0) [last]", []).append((s[roles["l0"] & m, 0, 1].max() - t0) / 100.0)
        f.setdefault("chain seen(0) [last]", []).append((s[chain & m, 0, 1].max() - t0) / 100.0)
        f.setdefault("chain bwd_pub(0) [median]", []).append((np.median(s[chain & m, 0, ref_k]) - t0) / 100.0)
        f.setdefault("chain bwd_pub(1) [median]", []).append((np.median(s[chain & m, 1, ref_k]) - t0) / 100.0)
    print("fill (us from the first layer-0 stamp, median over replicas):",
          {k: round(float(np.median(v)), 2) for k, v in f.items()})
    ends = [np.median(s[chain, i, ref_k]) for i in range(min(8, nst))]
    d = np.diff([x for x in ends if x > 0]) / 100.0
    print("step period (us):", np.round(d, 2), "median", np.round(np.median(d), 2) if len(d) else None)


if __name__ == "__main__":
    main()
