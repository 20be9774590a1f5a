"""Reference training engine on torch tensors (CPU, or GPU for custom ops).

This is the semantic anchor of the framework: it runs
the model's layer chain op by op with autograd, applies the Keras 2.10
optimizer rules from ``models/optimizers.py`` and the loss/metric formulas from
``models/losses.py``/``metrics.py``.  It handles everything the native
executor does not fuse (custom activation/loss/metric callables, stacked
activations, Adadelta/Nadam, ...), and the HIP kernels are tested against it.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models import activations as A
from ..models import optimizers as O
from ..models.layers import Activation, Dense, Dropout, Flatten
from .plan import flatten_weights, unflatten_weights
from .trainer import TrainerBase, prepare_features, prepare_targets, split_point


class _Bf16OperandMatmul(torch.autograd.Function):
    """fp32 x @ w with every matrix-core operand rounded to bf16 -- x and w forward, the
    incoming gradient and the other operand in both backward products -- and fp32
    products / sums: the arithmetic of the native engine's mixed_bfloat16 kernels
    (bf16 MFMA operands, fp32 accumulation, fp32 masters), as a reference for them."""

    @staticmethod
    def forward(ctx, x, w):
        xr, wr = x.bfloat16().float(), w.bfloat16().float()
        ctx.save_for_backward(xr, wr)
        return xr @ wr

    @staticmethod
    def backward(ctx, g):
        xr, wr = ctx.saved_tensors
        gr = g.bfloat16().float()
        return gr @ wr.t(), xr.t() @ gr


class TorchTrainer(TrainerBase):
    def __init__(self, model, plan, R: int = 1, batch_size: int = 32, device=None, seed: Optional[int] = None,
                 hash_dropout_seed: Optional[int] = None, bf16_operands: bool = False):
        super().__init__(model, plan, R, batch_size)
        # True: every Dense product takes bf16-rounded operands (_Bf16OperandMatmul), the
        # fp32 reference of the mixed_bfloat16 native kernels
        self.bf16_operands = bool(bf16_operands)
        # None: dropout masks from torch's generator; an int: the native engine's
        # counter-hash masks for that executor seed (ops/dropout_hash.py), so the two
        # engines can be compared step for step with dropout on
        self.hash_dropout_seed = hash_dropout_seed
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.like = model.get_weights()
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(int(seed) if seed is not None else int(np.random.randint(0, 2**31 - 1)))
        self.opts = [O.clone(model.optimizer) for _ in range(self.R)]
        self.params: List[List[torch.Tensor]] = []
        self.state = []
        self.iters = [0] * self.R
        self.set_weights_flat(flatten_weights(self.like))
        self.xs = self.ys = None

    # ---------------------------------------------------------------- weights
    def set_weights_flat(self, flat):
        flat = np.asarray(flat, np.float32)
        if flat.ndim == 1:
            flat = np.broadcast_to(flat, (self.R, flat.size))
        # like keras set_weights: the optimizer state (moments, iteration) is kept
        fresh = not getattr(self, "params", None)
        if fresh:
            self.params = []
        for r in range(self.R):
            ws = unflatten_weights(flat[r], self.like)
            if fresh:
                self.params.append([torch.tensor(w, device=self.device) for w in ws])
            else:
                for p, w in zip(self.params[r], ws):
                    p.copy_(torch.from_numpy(np.ascontiguousarray(w)).to(p.device))
        if fresh:
            self.state = [opt.init_state(p) for opt, p in zip(self.opts, self.params)]

    def get_weights_flat(self):
        return np.stack([np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in ps]) for ps in self.params])

    def get_state_flat(self):
        k = self.opts[0].n_state() if self.opts else 0
        out = np.zeros((self.R, max(k, 1), sum(p.numel() for p in self.params[0])), np.float32)
        for r in range(self.R):
            for j in range(k):
                out[r, j] = np.concatenate([s[j].detach().cpu().numpy().reshape(-1) for s in self.state[r]])
        return out, np.asarray(self.iters, np.int64)

    def set_state_flat(self, state, iterations):
        state = np.asarray(state, np.float32)
        k = self.opts[0].n_state() if self.opts else 0
        for r in range(self.R):
            for j in range(k):
                off = 0
                for s in self.state[r]:
                    n = s[j].numel()
                    s[j].copy_(torch.from_numpy(state[r, j, off:off + n].reshape(s[j].shape)).to(s[j].device))
                    off += n
        self.iters = [int(i) for i in np.broadcast_to(np.asarray(iterations), (self.R,))]

    def reset_optimizer_state(self):
        self.state = [opt.init_state(p) for opt, p in zip(self.opts, self.params)]
        self.iters = [0] * self.R

    # ---------------------------------------------------------------- forward
    def forward(self, r: int, x: torch.Tensor, training: bool, ps=None):
        h = x
        wi = 0
        dense = -1  # index of the Dense layer whose output the ops act on (the kernels' `layer`)
        pre, last_act = None, None
        ps = self.params[r] if ps is None else ps
        for op in self.plan.ops:
            if isinstance(op, Dense):
                dense += 1
                h = _Bf16OperandMatmul.apply(h, ps[wi]) if self.bf16_operands else h @ ps[wi]
                wi += 1
                if op.use_bias:
                    h = h + ps[wi]
                    wi += 1
                pre, last_act = h, op.activation
                h = op.activation(h)
            elif isinstance(op, Activation):
                pre, last_act = h, op.activation
                h = op.activation(h)
            elif isinstance(op, Dropout):
                if training and op.rate > 0:
                    if self.hash_dropout_seed is not None:
                        from .dropout_hash import keep_mask
                        keep = torch.from_numpy(keep_mask(self.hash_dropout_seed, r, dense, self.iters[r],
                                                          h.shape[0], h.shape[1], op.rate)).to(h.device)
                    else:
                        keep = torch.rand(h.shape, generator=self.gen).to(h.device) >= op.rate
                    h = h * keep.to(h.dtype) / (1.0 - op.rate)
            elif isinstance(op, Flatten):
                h = h.reshape(h.shape[0], -1)
        logits = None
        if last_act is A.softmax and self.loss.name in ("categorical_crossentropy", "sparse_categorical_crossentropy"):
            logits = pre
        elif last_act is A.sigmoid and self.loss.name == "binary_crossentropy":
            logits = pre
        return h, logits

    def _metric_logits(self, m, last_logits):
        return last_logits

    def _loss_and_metrics(self, y, pred, logits):
        per = self.loss(y, pred, logits)
        if per.dim() > 1:
            per = per.reshape(per.shape[0], -1).mean(-1)
        mvals = []
        for m in self.metrics:
            v = m(y, pred, logits)
            if v.dim() > 1:
                v = v.reshape(v.shape[0], -1).mean(-1)
            mvals.append(v)
        return per, mvals

    # ------------------------------------------------------------------- data
    def set_data(self, xs, ys, validation_split=0.0, active=None, shuffle=True):
        assert len(xs) == self.R and len(ys) == self.R
        self.xs, self.ys, self.split, self.active = [], [], [], []
        self.shuffle = shuffle
        for r in range(self.R):
            x = prepare_features(xs[r], self.in_dim) if len(xs[r]) else np.zeros((0, self.in_dim), np.float32)
            y = prepare_targets(ys[r], self.n_out, self.loss) if len(ys[r]) else np.zeros((0, 1), np.float32)
            self.xs.append(torch.tensor(x, device=self.device))
            self.ys.append(torch.tensor(y, device=self.device))
            self.split.append(split_point(len(x), validation_split))
            self.active.append(True if active is None else bool(active[r]))

    # ------------------------------------------------------------------ train
    def train_batch(self, r: int, xb: torch.Tensor, yb: torch.Tensor):
        ps = self.params[r]
        for p in ps:
            p.requires_grad_(True)
        pred, logits = self.forward(r, xb, True)
        per, mvals = self._loss_and_metrics(yb, pred, logits)
        loss = per.mean()
        grads = torch.autograd.grad(loss, ps, allow_unused=True)
        grads = [g if g is not None else torch.zeros_like(p) for g, p in zip(grads, ps)]
        for p in ps:
            p.requires_grad_(False)
        self.opts[r].apply_torch(ps, grads, self.state[r], self.iters[r])
        self.iters[r] += 1
        return per.detach(), [m.detach() for m in mvals]

    def _grads(self, r, xb, yb):
        ps = self.params[r]
        for p in ps:
            p.requires_grad_(True)
        pred, logits = self.forward(r, xb, True)
        per, mvals = self._loss_and_metrics(yb, pred, logits)
        grads = torch.autograd.grad(per.mean(), ps, allow_unused=True)
        for p in ps:
            p.requires_grad_(False)
        grads = [g if g is not None else torch.zeros_like(p) for g, p in zip(grads, ps)]
        return torch.cat([g.reshape(-1) for g in grads]), per.detach(), [m.detach() for m in mvals]

    def fit_allreduce(self, epochs, allreduce, verbose=0):
        """Per-step synchronous DP: every replica computes its batch gradient, the
        [R, n] gradient block goes through ``allreduce`` (which leaves the
        averaged gradient in every row), then every replica applies it."""
        hist = [dict() if self.active[r] else None for r in range(self.R)]
        shapes = [p.shape for p in self.params[0]]
        sizes = [p.numel() for p in self.params[0]]
        for epoch in range(int(epochs)):
            idx = [torch.randperm(self.split[r], generator=self.gen) if self.shuffle else torch.arange(self.split[r])
                   for r in range(self.R)]
            steps = max([int(math.ceil(self.split[r] / self.B)) for r in range(self.R) if self.active[r]] or [0])
            sums = [np.zeros(2 + len(self.metrics)) for _ in range(self.R)]
            for s in range(steps):
                G = torch.zeros(self.R, sum(sizes), device=self.device)
                has = []
                for r in range(self.R):
                    bi = idx[r][s * self.B:(s + 1) * self.B]
                    if not self.active[r] or len(bi) == 0:
                        has.append(False)
                        continue
                    bi = bi.to(self.device)
                    G[r], per, mvals = self._grads(r, self.xs[r][bi], self.ys[r][bi])
                    has.append(True)
                    sums[r][0] += float(per.sum())
                    sums[r][1] += per.numel()
                    for i, v in enumerate(mvals):
                        sums[r][2 + i] += float(v.sum())
                allreduce(G)
                for r in range(self.R):
                    if has[r]:
                        grads = [g.reshape(sh) for g, sh in zip(torch.split(G[r], sizes), shapes)]
                        self.opts[r].apply_torch(self.params[r], grads, self.state[r], self.iters[r])
                        self.iters[r] += 1
            for r in range(self.R):
                if not self.active[r]:
                    continue
                n = self.split[r]
                h = self._history_from_sums(sums[r]) if n > 0 else {}
                if len(self.xs[r]) - n > 0:
                    h.update(self._history_from_sums(self._eval_tensors(r, self.xs[r][n:], self.ys[r][n:]), "val_"))
                for k, v in h.items():
                    hist[r].setdefault(k, []).append(v)
                if verbose:
                    self.print_epoch(epoch, epochs, h, r)
        return hist

    def fit(self, epochs, verbose=0, allreduce=None):
        if allreduce is not None:
            return self.fit_allreduce(epochs, allreduce, verbose)
        hist = [dict() if self.active[r] else None for r in range(self.R)]
        for epoch in range(int(epochs)):
            for r in range(self.R):
                if not self.active[r]:
                    continue
                n = self.split[r]
                idx = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
                sums = np.zeros(2 + len(self.metrics))
                for b0 in range(0, n, self.B):
                    bi = idx[b0:b0 + self.B].to(self.device)
                    per, mvals = self.train_batch(r, self.xs[r][bi], self.ys[r][bi])
                    sums[0] += float(per.sum())
                    sums[1] += per.numel()
                    for i, v in enumerate(mvals):
                        sums[2 + i] += float(v.sum())
                h = self._history_from_sums(sums) if n > 0 else {}
                nval = len(self.xs[r]) - n
                if nval > 0:
                    ev = self._eval_tensors(r, self.xs[r][n:], self.ys[r][n:])
                    h.update(self._history_from_sums(ev, "val_"))
                for k, v in h.items():
                    hist[r].setdefault(k, []).append(v)
                if verbose:
                    self.print_epoch(epoch, epochs, h, r)
        return hist

    def train_steps(self, nsteps: int):
        """Bench helper: nsteps batches per replica over the (shuffled) shard."""
        for r in range(self.R):
            n = self.split[r]
            for s in range(nsteps):
                b0 = (s * self.B) % max(n, 1)
                self.train_batch(r, self.xs[r][b0:b0 + self.B], self.ys[r][b0:b0 + self.B])

    # ------------------------------------------------------------------- eval
    @torch.no_grad()
    def _eval_tensors(self, r, x, y, bs=None):
        bs = bs or max(self.B, 1024)
        sums = np.zeros(2 + len(self.metrics))
        for b0 in range(0, len(x), bs):
            pred, logits = self.forward(r, x[b0:b0 + bs], False)
            per, mvals = self._loss_and_metrics(y[b0:b0 + bs], pred, logits)
            sums[0] += float(per.sum())
            sums[1] += per.numel()
            for i, v in enumerate(mvals):
                sums[2 + i] += float(v.sum())
        return sums

    def evaluate_sums(self, x, y, batch_size=None, r: int = 0) -> np.ndarray:
        xt = torch.tensor(prepare_features(x, self.in_dim), device=self.device)
        yt = torch.tensor(prepare_targets(y, self.n_out, self.loss), device=self.device)
        return self._eval_tensors(r, xt, yt, batch_size)

    def evaluate(self, x, y, batch_size=None, r: int = 0):
        s = self.evaluate_sums(x, y, batch_size, r)
        cnt = max(s[1], 1.0)
        return [float(s[0] / cnt)] + [float(v / cnt) for v in s[2:]]

    @torch.no_grad()
    def predict(self, x, batch_size=None, r: int = 0):
        # Row results must not depend on how rows are batched (reference
        # tests/test_ml_model.py:345-354 requires batched == unbatched inference
        # exactly): BLAS kernels pick blockings by M, so inference runs in fp64
        # and rounds to fp32 once, which makes every row's value batch-invariant.
        xt = torch.tensor(prepare_features(x, self.in_dim), device=self.device, dtype=torch.float64)
        ps = [p.detach().double() for p in self.params[r]]
        bs = batch_size or 4096
        outs = [self.forward(r, xt[b0:b0 + bs], False, ps)[0].float() for b0 in range(0, len(xt), bs)]
        if not outs:
            return np.zeros((0, self.n_out), np.float32)
        return torch.cat(outs).float().cpu().numpy()

    def train_on_batch(self, x, y, r: int = 0):
        xt = torch.tensor(prepare_features(x, self.in_dim), device=self.device)
        yt = torch.tensor(prepare_targets(y, self.n_out, self.loss), device=self.device)
        per, mvals = self.train_batch(r, xt, yt)
        return [float(per.mean())] + [float(v.mean()) for v in mvals]
