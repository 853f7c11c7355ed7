"""Dense layer — mirror of torchrec/model/layer/Dense.py:4-24.

Linear -> ReLU -> Dropout.  As in the reference, ReLU is applied whatever the
``activation`` string says (Dense.py:14-17).  On a GPU the Linear + bias + ReLU
run as one MFMA GEMM with a fused epilogue (``pytorchrec_amd.dense``); the
``linear`` submodule keeps the reference's parameter names and init.
"""
from torch.nn import Dropout, Linear, Module

from pytorchrec_amd import dense as dense_ops


class Dense(Module):
    def __init__(self, input_units: int, output_units: int, activation: str, dropout: float):
        super().__init__()
        self.linear = Linear(input_units, output_units)
        self.activation_name = activation  # reference: always ReLU
        self.dropout = Dropout(dropout)

    def forward(self, x):
        x = dense_ops.linear(x, self.linear.weight, self.linear.bias, act="relu")
        return self.dropout(x) if self.dropout.p > 0 and self.training else x
