"""MLP — mirror of torchrec/model/layer/MLP.py:8-23 (stack of Dense layers named
``dense_{i}`` inside ``self.mlp``, so state_dict keys match the reference)."""
from typing import List

from torch.nn import Module, Sequential

from pytorchrec_amd.model.layer.Dense import Dense


class MLP(Module):
    def __init__(self, input_units: int, hidden_units_list: List[int], activation: str,
                 dropout: float):
        super().__init__()
        self.mlp = Sequential()
        pre = input_units
        for i, units in enumerate(hidden_units_list):
            self.mlp.add_module(f"dense_{i}", Dense(pre, units, activation, dropout))
            pre = units
        self.output_units = pre

    def forward(self, x):
        return self.mlp(x)
