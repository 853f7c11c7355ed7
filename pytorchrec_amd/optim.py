"""Optimizers: the reference's ``torchrec.optim`` surface plus row-wise Adagrad.

Mirrors ``torchrec/optim/optimizers.py:7-20`` (registry ``get_optimizer`` of
"sgd" / "adam" / "adamw") and ``torchrec/optim/AdamW.py:8-61`` (AdamW with
``correct_bias``, decoupled weight decay applied after the step, eps added to
sqrt(v) before the bias-corrected step size).  ``RowWiseAdagrad`` is the
recsys-standard low-memory Adagrad (one accumulator per embedding row) that
SURVEY.md §8(f) rank 3 asks for; it has no reference counterpart.

Dense parameters step here in torch.  Embedding banks never do: ``IModel.compile``
hands the matching fused row-sparse update to the bank (include/mrec.h
MREC_BWD_ADAGRAD / _ROWWISE_ADAGRAD / _ADAM), which reads its hyper-parameters
from the optimizer's param group (``fused_spec``).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Type

import torch
from torch.optim import SGD, Adam, Adagrad
from torch.optim.optimizer import Optimizer


class AdamW(Optimizer):
    """The reference AdamW (torchrec/optim/AdamW.py:8-61): same arguments, defaults,
    checks and update order."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0,
                 correct_bias=True):
        if lr < 0.0:
            raise ValueError("Invalid learning rate: {} - should be >= 0.0".format(lr))
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError("Invalid beta parameter: {} - should be in [0.0, 1.0[".format(betas[0]))
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameter: {} - should be in [0.0, 1.0[".format(betas[1]))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {} - should be >= 0.0".format(eps))
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      correct_bias=correct_bias))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad
                if grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients, please consider "
                                       "SparseAdam instead")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                m, v = state["exp_avg"], state["exp_avg_sq"]
                state["step"] += 1
                m.mul_(beta1).add_(grad, alpha=1.0 - beta1)
                v.mul_(beta2).addcmul_(grad, grad, value=1.0 - beta2)
                denom = v.sqrt().add_(group["eps"])
                step_size = group["lr"]
                if group["correct_bias"]:
                    step_size = (step_size * math.sqrt(1.0 - beta2 ** state["step"])
                                 / (1.0 - beta1 ** state["step"]))
                p.addcdiv_(m, denom, value=-step_size)
                if group["weight_decay"] > 0.0:
                    p.add_(p, alpha=-group["lr"] * group["weight_decay"])
        return loss


class RowWiseAdagrad(Optimizer):
    """Adagrad with one accumulator per row of a 2-D parameter (the mean of the
    row's squared gradient is accumulated; 1-D parameters are element-wise):
    s_r += mean_d g_rd^2,  w_rd -= lr * g_rd / (sqrt(s_r) + eps).  An embedding
    bank's first-order weight keeps its own accumulator per row."""

    def __init__(self, params, lr=1e-2, eps=1e-10):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if eps < 0.0:
            raise ValueError(f"Invalid epsilon value: {eps}")
        super().__init__(params, dict(lr=lr, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                state = self.state[p]
                if len(state) == 0:
                    shape = (p.shape[0], 1) if p.dim() == 2 else p.shape
                    state["sum"] = torch.zeros(shape, dtype=torch.float32, device=p.device)
                s = state["sum"]
                if p.dim() == 2:
                    s.add_((g.float() ** 2).mean(dim=1, keepdim=True))
                else:
                    s.add_(g.float() ** 2)
                p.add_((g.float() / (s.sqrt() + group["eps"])).to(p.dtype), alpha=-group["lr"])
        return loss


_optimizer_classes: Dict[str, Type[Optimizer]] = {
    "sgd": SGD,
    "adam": Adam,
    "adamw": AdamW,
    "adagrad": Adagrad,
    "rowwise_adagrad": RowWiseAdagrad,
}

optimizer_name_list = _optimizer_classes.keys()


def get_optimizer(optimizer_name: str) -> Type[Optimizer]:
    """Optimizer class by name (reference optimizers.py:16-20, same error)."""
    if (not isinstance(optimizer_name, str)) or (optimizer_name not in _optimizer_classes):
        raise ValueError(f"optimizer_name参数不合法: {optimizer_name}")
    return _optimizer_classes[optimizer_name]


def fused_spec(optimizer: Optimizer, group: dict) -> Optional[dict]:
    """The fused row-sparse update equivalent to ``optimizer`` on an embedding bank
    in ``group`` (keyword arguments of ``EmbeddingBank.use_fused_optimizer`` plus
    ``kind``), or None when there is none (the bank then keeps a dense gradient)."""
    if group.get("maximize", False):
        return None
    if isinstance(optimizer, Adagrad):
        if (group.get("lr_decay", 0) != 0 or group.get("weight_decay", 0) != 0
                or group.get("initial_accumulator_value", 0) != 0):
            return None  # rows not looked up would still move (decay) / differ at start
        return dict(kind="adagrad", eps=group["eps"])
    if isinstance(optimizer, RowWiseAdagrad):
        return dict(kind="rowwise_adagrad", eps=group["eps"])
    if isinstance(optimizer, AdamW):
        return dict(kind="adam", eps=group["eps"], betas=group["betas"],
                    weight_decay=group.get("weight_decay", 0.0), decoupled=True,
                    bias_correction=bool(group.get("correct_bias", True)))
    if type(optimizer) is Adam:
        if group.get("amsgrad", False):
            return None
        if group.get("decoupled_weight_decay", False) and group.get("weight_decay", 0.0) != 0:
            # torch >= 2.6 Adam(decoupled_weight_decay=True) decays p by lr*wd BEFORE the
            # moment update; the fused kernel's decoupled order is the reference AdamW's
            # (decay after the step, AdamW.py:53-59): keep the dense gradient instead
            return None
        return dict(kind="adam", eps=group["eps"], betas=group["betas"],
                    weight_decay=group.get("weight_decay", 0.0), decoupled=False)
    return None
