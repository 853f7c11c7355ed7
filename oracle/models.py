"""torch-CPU restatement of the reference training path for the CTR models
(TEST INFRASTRUCTURE ONLY: checker + bench.py's cpu_baseline leg).

Built exactly from the reference's primitives, the way a PyTorchRec user would
write these models on the reference:
  * one ``torch.nn.Embedding(rows_f, D)`` per field (FunkSVD.py:39-41) and one
    ``Embedding(rows_f, 1)`` first-order bias per field (SVDPP.py:40-41), dense
    gradients (``sparse=False``) -> ``aten::embedding_dense_backward``;
  * reference ``MLP`` semantics: Linear -> ReLU per layer (MLP.py:8-23, Dense.py);
  * init normal(0, 0.01) (IModel._reset_weights_fn, IModel.py:61-68);
  * step = forward -> BCEWithLogits -> zero_grad -> backward -> SGD.step over ALL
    parameters, i.e. ``IModel.train_step`` (IModel.py:116-125).

``dtype=torch.float64`` gives the model-level parity oracle; float32 is the CPU
baseline (SURVEY.md §8(d) "CPU baseline").
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch import nn


def _reset(m):
    if isinstance(m, (nn.Linear, nn.Embedding)):
        nn.init.normal_(m.weight, 0.0, 0.01)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.normal_(m.bias, 0.0, 0.01)


def _mlp(units: Sequence[int]) -> nn.Sequential:
    layers = []
    for a, b in zip(units[:-1], units[1:]):
        layers += [nn.Linear(a, b), nn.ReLU()]
    return nn.Sequential(*layers)


class RefDeepFM(nn.Module):
    """DeepFM the reference way.  ``deep=False`` gives FM (config C1).

    ``bf16_points=True`` is NOT the reference: the same model with every tensor the
    MI355X tower stores in bf16 rounded there (x0 = [v | dense], the MLP weights as
    MFMA operands, each hidden activation, and the gradients at the same points:
    dh_l, dx0; fp32 accumulation; the FM / first-order terms and the output layer's
    weights stay fp32).  The C2 parity test sizes its bar by this model's distance
    to the fp64 one."""

    def __init__(self, category_nums: List[int], n_dense: int, emb_size: int = 16,
                 layers=(400, 400, 400), deep: bool = True, dtype=torch.float32, seed: int = 2020,
                 bf16_points: bool = False):
        super().__init__()
        torch.manual_seed(seed)
        self.F, self.D, self.n_dense = len(category_nums), emb_size, n_dense
        self.emb = nn.ModuleList([nn.Embedding(n, emb_size) for n in category_nums])
        self.w1 = nn.ModuleList([nn.Embedding(n, 1) for n in category_nums])
        self.dense_w = nn.Linear(n_dense, 1, bias=False) if n_dense else None
        self.global_bias = nn.Parameter(torch.zeros(1))
        self.deep = deep
        self.bf16_points = bf16_points
        if deep:
            self.mlp = _mlp([self.F * emb_size + n_dense, *layers])
            self.out = nn.Linear(layers[-1], 1)
        self.apply(_reset)
        self.to(dtype)

    def forward(self, ids: torch.Tensor, dense: torch.Tensor | None):
        """ids [B, F] int64, dense [B, n_dense] -> logits [B]."""
        v = torch.stack([e(ids[:, f]) for f, e in enumerate(self.emb)], 1)  # [B, F, D]
        s = v.sum(1)
        logit = 0.5 * (s * s - (v * v).sum(1)).sum(-1)
        logit = logit + torch.cat([w(ids[:, f]) for f, w in enumerate(self.w1)], 1).sum(1)
        logit = logit + self.global_bias
        if self.dense_w is not None:
            logit = logit + self.dense_w(dense).squeeze(-1)
        if self.deep:
            x0 = torch.cat([v.reshape(v.shape[0], -1)] + ([dense] if self.n_dense else []), 1)
            if not self.bf16_points:
                return logit + self.out(self.mlp(x0)).squeeze(-1)
            x = _rb(x0)
            for m in self.mlp:
                if isinstance(m, nn.Linear):
                    x = _rb(torch.relu(x @ _rbv(m.weight).T + m.bias))
            logit = logit + (x @ self.out.weight.T + self.out.bias).squeeze(-1)
        return logit


class _RoundBF16(torch.autograd.Function):
    """Identity that rounds its value (forward) and its gradient (backward) to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _rb(x):
    return _RoundBF16.apply(x)


class _RoundBF16Value(torch.autograd.Function):
    """Rounds the value to bf16, passes the gradient through unrounded (a weight
    read as a bf16 MFMA operand whose gradient is accumulated and kept in fp32)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


def _rbv(x):
    return _RoundBF16Value.apply(x)


class RefDCNv2(nn.Module):
    """Stacked DCN-v2 the reference way (cross layers = nn.Linear(d, d)).

    ``bf16_points=True`` is NOT the reference: the same model with every tensor the
    MI355X path stores in bf16 rounded there (x0, the cross outputs, MLP
    activations, the weights as GEMM operands, and the gradients at the same
    points; fp32 accumulation).  Its distance to the fp64 model is what bf16
    storage alone costs — the parity tests use it to size their tolerance."""

    def __init__(self, category_nums: List[int], n_dense: int, emb_size=16, n_cross=3,
                 layers=(400, 400), dtype=torch.float32, seed=2020, bf16_points=False):
        super().__init__()
        torch.manual_seed(seed)
        self.emb = nn.ModuleList([nn.Embedding(n, emb_size) for n in category_nums])
        d = len(category_nums) * emb_size + n_dense
        self.cross = nn.ModuleList([nn.Linear(d, d) for _ in range(n_cross)])
        self.mlp = _mlp([d, *layers])
        self.out = nn.Linear(layers[-1], 1)
        self.bf16_points = bf16_points
        self.apply(_reset)
        self.to(dtype)

    def forward(self, ids, dense):
        v = torch.cat([e(ids[:, f]) for f, e in enumerate(self.emb)], 1)
        x0 = torch.cat([v, dense], 1) if dense is not None else v
        if not self.bf16_points:
            x = x0
            for c in self.cross:
                x = x0 * c(x) + x
            return self.out(self.mlp(x)).squeeze(-1)
        lin = (lambda x, m: x @ _rb(m.weight).T + m.bias)
        x0 = _rb(x0)
        x = x0
        for c in self.cross:
            x = _rb(x0 * lin(x, c) + x)
        for m in self.mlp:
            if isinstance(m, nn.Linear):
                x = _rb(torch.relu(lin(x, m)))
        return (x @ self.out.weight.T + self.out.bias).squeeze(-1)


class _RoundBF16Grad(torch.autograd.Function):
    """Passes the value unrounded, rounds the gradient to bf16 (a pre-activation
    whose gradient the MI355X path stores as a bf16 MFMA operand while the value
    itself never leaves fp32 registers)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _rbg(x):
    return _RoundBF16Grad.apply(x)


class RefDIN(nn.Module):
    """DIN (config C4) the reference way.  The reference has no DIN; this is built
    from its primitives, which is what a PyTorchRec user would write:

      * an item and a category ``nn.Embedding`` shared by the target and the
        history (FunkSVD.py:39-41), init normal(0, 0.01) (IModel.py:61-68);
        q = [item(iid) | cate(cid)], k_j = [item(his_j) | cate(hcat_j)];
      * history validity ``his > 0`` with position 0 forced valid
        (``get_valid_his_index``, torchrec/model/utils.py:5-10);
      * attention unit = reference ``MLP`` (Linear -> ReLU, MLP.py:8-23) over
        [q, k, q - k, q * k] + Linear(h, 1) -> scores;
      * masked softmax: -inf on invalid keys, then softmax over the history
        (``scaled_dot_product_attention``, SASRec.py:14-31; its global-max shift is
        a no-op for softmax and is kept for fidelity), pooled u = sum_j a_j k_j
        (the weighted-sum form of SASRec.py:30 / SVDPP.py:49-55);
      * top = MLP over [q, u] + Linear(last, 1) -> logit (NCF.py:68-74).

    ``bf16_points=True`` is NOT the reference: the same model with every tensor
    the MI355X path stores in bf16 rounded there: the
    attention-unit input's q - k and q * k, W1 / W2 as MFMA operands, H1 (value)
    and the layer-1 / layer-2 pre-activation gradients (dZ1, dZ2), the pooled u
    (top = [q | u] is a bf16 tensor, and so is its gradient), the top tower as in
    RefDeepFM, and each gathered row's gradient (one bf16 value per lookup).  H2,
    the scores, the softmax and w3 stay fp32.  Its distance to the fp64 model is
    what bf16 storage alone costs; the C4 parity test sizes its bar by it."""

    def __init__(self, item_rows: int, cate_rows: int, emb_size: int = 16, att_layers=(80, 40),
                 layers=(200, 80), dtype=torch.float32, seed: int = 2020,
                 bf16_points: bool = False):
        super().__init__()
        torch.manual_seed(seed)
        E = 2 * emb_size
        self.item = nn.Embedding(item_rows, emb_size)
        self.cate = nn.Embedding(cate_rows, emb_size)
        self.att_mlp = _mlp([4 * E, *att_layers])
        self.att_out = nn.Linear(att_layers[-1], 1)
        self.mlp = _mlp([2 * E, *layers])
        self.out = nn.Linear(layers[-1], 1)
        self.bf16_points = bf16_points
        self.apply(_reset)
        self.to(dtype)

    def forward(self, iid, cid, his, hcat):
        """iid / cid [B], his / hcat [B, L] int64 -> logits [B]."""
        B, L = his.shape
        rb = self.bf16_points
        q = torch.cat([self.item(iid), self.cate(cid)], -1)                   # [B, E]
        k = torch.cat([self.item(his), self.cate(hcat)], -1)                  # [B, L, E]
        if rb:  # one bf16 gradient per gathered row
            q, k = _rb(q), _rb(k)
        valid = his.gt(0)
        valid[:, 0] = True
        qb = q[:, None, :].expand_as(k)
        if rb:
            x = torch.cat([qb, k, _rbv(qb - k), _rbv(qb * k)], -1)
        else:
            x = torch.cat([qb, k, qb - k, qb * k], -1)
        lins = [m for m in self.att_mlp if isinstance(m, nn.Linear)]
        for i, m in enumerate(lins):
            if not rb:
                x = torch.relu(m(x))
                continue
            z = _rbg(x @ _rbv(m.weight).T + m.bias)
            x = torch.relu(z)
            if i + 1 < len(lins):
                x = _rbv(x)  # H1 is a bf16 MFMA operand; H2 stays fp32
        s = self.att_out(x).squeeze(-1)                                       # [B, L]
        # SASRec.py:26 (the shift's gradient is analytically zero; detached so it
        # does not leak rounding noise into whichever row holds the max)
        s = s - s.detach().max()
        a = s.masked_fill(~valid, float("-inf")).softmax(-1)
        u = (a[..., None] * k).sum(1)
        top = torch.cat([q, u], -1)
        if not rb:
            return self.out(self.mlp(top)).squeeze(-1)
        x = _rb(top)
        for m in self.mlp:
            if isinstance(m, nn.Linear):
                x = _rb(torch.relu(x @ _rbv(m.weight).T + m.bias))
        return (x @ self.out.weight.T + self.out.bias).squeeze(-1)


def din_batch(item_rows: int, cate_rows: int, batch: int, L: int = 50, seed: int = 0):
    """SURVEY.md §8(d) C4 synthetic batch (bench.din_batch's recipe): ids uniform
    over the non-PAD rows, history lengths U{1..L}, tail-padded with 0
    (interaction_history_list.py:17-29), labels Bernoulli(0.25)."""
    g = torch.Generator().manual_seed(seed)
    iid = torch.randint(1, item_rows, (batch,), generator=g)
    cid = torch.randint(1, cate_rows, (batch,), generator=g)
    his = torch.randint(1, item_rows, (batch, L), generator=g)
    hcat = torch.randint(1, cate_rows, (batch, L), generator=g)
    lens = torch.randint(1, L + 1, (batch, 1), generator=g)
    pad = torch.arange(L)[None, :] >= lens
    his[pad] = 0
    hcat[pad] = 0
    label = (torch.rand(batch, generator=g) < 0.25).float()
    return iid, cid, his, hcat, label


def sgd_train_step(model: nn.Module, opt: torch.optim.Optimizer, ids, dense, label):
    """``IModel.train_step`` (IModel.py:116-125) with BCEWithLogitsLoss."""
    logit = model(*ids) if isinstance(ids, (tuple, list)) else model(ids, dense)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, label.to(logit.dtype))
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss


def criteo_batch(category_nums, batch: int, n_dense: int = 13, seed: int = 0, zipf: float = 0.0,
                 label_rate: float = 0.25):
    """SURVEY.md §8(d) synthetic Criteo-shaped batch: ids uniform (seed 0) or Zipf
    (seed 1), dense U[0,1) (seed 2), labels Bernoulli(0.25) (seed 3)."""
    import numpy as np
    F = len(category_nums)
    rng = np.random.default_rng(seed)
    if zipf:  # truncated Zipf over each table's rows (inverse CDF), as bench.zipf_ids
        def trunc(n):
            cdf = np.cumsum(np.arange(1, n + 1, dtype=np.float64) ** -zipf)
            return np.minimum(np.searchsorted(cdf / cdf[-1], rng.random(batch), side="right"), n - 1)
        ids = np.stack([trunc(n) for n in category_nums], 1)
    else:
        ids = np.stack([rng.integers(0, n, batch) for n in category_nums], 1)
    dense = np.random.default_rng(seed + 2).random((batch, n_dense), dtype=np.float32)
    label = (np.random.default_rng(seed + 3).random(batch) < label_rate).astype(np.float32)
    return (torch.from_numpy(ids.astype(np.int64)), torch.from_numpy(dense),
            torch.from_numpy(label))
