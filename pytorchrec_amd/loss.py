"""Losses — the CTR loss the reference registry lacks (torchrec/loss/losses.py:8-21
registers BPR / Top1 / MSE only).

``BCEWithLogitsLoss`` is a ``torch.nn.modules.loss._Loss`` (so it passes
``IModel.compile``'s type check, IModel.py:103-104) with exactly
``torch.nn.BCEWithLogitsLoss(reduction="mean")`` semantics; on a GPU its forward
and backward are single libmrec kernels (fixed-order reduction).
"""
from typing import Dict, Type

import torch
from torch.nn.modules.loss import _Loss, MSELoss  # noqa

from pytorchrec_amd import _mrec


class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y):
        z = z.contiguous().float()
        y = y.contiguous().float()
        loss = torch.empty(1, dtype=torch.float32, device=z.device)
        _mrec.call("mrec_bce_fwd", z.data_ptr(), y.data_ptr(), z.numel(), loss.data_ptr(),
                   _mrec.stream_handle())
        ctx.save_for_backward(z, y)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        z, y = ctx.saved_tensors
        g = g.contiguous().float().reshape(1)
        dz = torch.empty_like(z)
        _mrec.call("mrec_bce_bwd", z.data_ptr(), y.data_ptr(), z.numel(), g.data_ptr(),
                   dz.data_ptr(), _mrec.stream_handle())
        return dz, None


class BCEWithLogitsLoss(_Loss):
    """Mean binary cross entropy on logits."""

    def __init__(self):
        super().__init__(reduction="mean")

    def forward(self, prediction, target):
        if prediction.is_cuda:
            return _BCEFn.apply(prediction.reshape(-1), target.reshape(-1))
        return torch.nn.functional.binary_cross_entropy_with_logits(prediction.float(),
                                                                    target.float())


_loss_classes: Dict[str, Type[_Loss]] = {
    "bce": BCEWithLogitsLoss,
    "mse": MSELoss,
}

loss_name_list = _loss_classes.keys()


def get_loss(loss_name: str) -> Type[_Loss]:
    """Mirror of torchrec/loss/losses.py:get_loss."""
    if (not isinstance(loss_name, str)) or (loss_name not in _loss_classes):
        raise ValueError(f"loss_name参数不合法: {loss_name}")
    return _loss_classes[loss_name]
