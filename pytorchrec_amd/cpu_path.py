"""The reference's own CPU path for an EmbeddingBank on a CPU device.

Config C1 of BASELINE.json runs FM through the CLI on the CPU ("PyTorch CPU path
(plumbing, no GPU)").  For a bank whose weight lives on the CPU, the ops in
``embedding.py`` dispatch here: plain torch ``index_select`` gathers and autograd
dense gradients, exactly the arithmetic ``nn.Embedding`` does on CPU
(FunkSVD.py:47-51, IModel.py:116-125).  This module is never used for a tensor on
a GPU — those go through libmrec or raise.
"""
from __future__ import annotations

from typing import List, Optional

import torch


def _rows(bank, ids: List[torch.Tensor]) -> List[torch.Tensor]:
    out = []
    for f, t in enumerate(ids):
        t = t.long()
        n = bank.category_nums[f]
        if t.numel() and (int(t.min()) < 0 or int(t.max()) >= n):
            raise IndexError("index out of range in self")
        out.append(t + bank.row_offset[f])
    return out


def _weight(bank):
    """The weight as seen by autograd: the parameter itself in dense mode; in fused
    SGD mode a detached leaf whose gradient is applied as SGD by a hook."""
    if bank.update == "dense" or not torch.is_grad_enabled():
        return bank.weight
    w = bank.weight.detach().requires_grad_()
    lr = bank.current_lr()
    target = bank.weight

    def _sgd(g):
        with torch.no_grad():
            target.add_(g.to(target.dtype), alpha=-lr)
        return g

    w.register_hook(_sgd)
    return w


def gather(bank, ids, out_dtype, with_w: bool):
    w = _weight(bank)
    rows = _rows(bank, ids)
    v = torch.cat([w.index_select(0, r)[:, :bank.dim] for r in rows], dim=1).to(out_dtype)
    if with_w:
        ww = torch.stack([w.index_select(0, r)[:, bank.dim] for r in rows], dim=1).float()
        return v, ww
    return v


def fm2(v: torch.Tensor) -> torch.Tensor:
    s = v.sum(dim=1)
    return 0.5 * (s * s - (v * v).sum(dim=1)).sum(dim=-1)


def interact(bank, ids, dense: Optional[torch.Tensor], dense_w, bias, use_fm2: bool,
             first_order: bool, x0_cols: int, x0_dtype):
    w = _weight(bank)
    rows = _rows(bank, ids)
    g = [w.index_select(0, r) for r in rows]
    return interact_rows(g, bank.dim, dense, dense_w, bias, use_fm2, first_order, x0_cols,
                         x0_dtype)


def interact_rows(g: List[torch.Tensor], dim: int, dense: Optional[torch.Tensor], dense_w, bias,
                  use_fm2: bool, first_order: bool, x0_cols: int, x0_dtype):
    """The interaction on already-gathered rows g[f] = [B, >= dim(+1)] (also the
    row-sharded CPU path, whose rows arrive through the exchange)."""
    v = torch.stack([x[:, :dim] for x in g], dim=1).float()  # [B, F, D]
    B = v.shape[0]
    logit = torch.zeros(B, dtype=torch.float32)
    if bias is not None:
        logit = logit + bias.float()
    if dense is not None and dense_w is not None:
        logit = logit + dense.float() @ dense_w.float()
    if use_fm2:
        logit = logit + fm2(v)
    if first_order:
        logit = logit + torch.stack([x[:, dim] for x in g], dim=1).float().sum(1)
    if not x0_cols:
        return logit
    parts = [v.reshape(B, -1)]
    if dense is not None:
        parts.append(dense.float())
    x0 = torch.cat(parts, dim=1)
    if x0.shape[1] < x0_cols:
        x0 = torch.nn.functional.pad(x0, (0, x0_cols - x0.shape[1]))
    return x0.to(x0_dtype), logit
