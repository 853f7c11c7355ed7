"""DCN-v2 (stacked): full-rank cross network then deep MLP (config C3).

Absent from the reference; built from its primitives:
embedding concat + dense features -> x0 (NCF.py:62-70 idiom), cross layers
x_{l+1} = x0 * (W_l x_l + b_l) + x_l with W_l an ``nn.Linear(d, d)`` (so the
reference init, IModel.py:61-66, applies), reference ``MLP`` on x_L, then
``Linear(last, 1)``.  On a GPU each cross layer is one MFMA GEMM with the
x0 * (.) + x_l epilogue fused.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import torch
from torch import Tensor
from torch.nn import Linear, ModuleList

from pytorchrec_amd import dense as dense_ops
from pytorchrec_amd.embedding import interact
from pytorchrec_amd.sharding import make_bank
from pytorchrec_amd.feature_column import CategoricalColumn, NumericColumn
from pytorchrec_amd.model.DeepFM import _CTRBase, _parse_layers, _round_up
from pytorchrec_amd.model.layer.MLP import MLP
from pytorchrec_amd.utils.argument import ArgumentDescription


class DCNv2(_CTRBase):
    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return [
            ArgumentDescription(name="emb_size", type_=int, help_info="embedding dim",
                                default_value=16, lower_closed_bound=1),
            ArgumentDescription(name="cross_layers", type_=int, help_info="number of cross layers",
                                default_value=3, lower_closed_bound=1),
            ArgumentDescription(name="layers", type_=str, help_info="deep MLP widths",
                                default_value="400,400"),
            ArgumentDescription(name="dropout", type_=float, help_info="MLP dropout",
                                default_value=0.0, lower_closed_bound=0.0, upper_open_bound=1.0),
        ]

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        super().check_argument_values(arguments)

    def __init__(self, sparse_columns: Sequence[CategoricalColumn],
                 dense_columns: Optional[Sequence[NumericColumn]] = None, label_column=None,
                 emb_size: int = 16, cross_layers: int = 3, layers=(400, 400),
                 dropout: float = 0.0, emb_dtype: torch.dtype = torch.float32, device=None,
                 **kwargs):
        self._setup_columns(sparse_columns, dense_columns, label_column, emb_size, emb_dtype,
                            device)
        self.n_cross = int(cross_layers)
        self.layers = _parse_layers(layers)
        self.dropout = float(dropout)
        super().__init__(**kwargs)

    def _init_weights(self):
        dev = self.build_device
        F, D, n = len(self.sparse_columns), self.emb_size, len(self.dense_columns)
        self.embeddings = make_bank([c.category_num for c in self.sparse_columns], D,
                                        with_first_order=False, dtype=self.emb_dtype, device=dev)
        self.deep_in = F * D + n
        self.x0_cols = _round_up(self.deep_in, 8)
        self.cross = ModuleList([Linear(self.deep_in, self.deep_in) for _ in range(self.n_cross)])
        self.mlp = MLP(self.deep_in, self.layers, "relu", self.dropout)
        self.prediction = Linear(self.layers[-1], 1)
        if dev is not None:
            for m in (self.cross, self.mlp, self.prediction):
                m.to(dev)

    def _x0(self, data: Dict[str, Tensor]):
        x0, _ = interact(self.embeddings, self._ids(data), self._dense(data), None, None,
                         fm2=False, first_order=False, x0_cols=self.x0_cols,
                         x0_dtype=self._x0_dtype())
        return x0

    def _cross(self, data: Dict[str, Tensor]):
        return dense_ops.cross_net(self._x0(data), [c.weight for c in self.cross],
                                   [c.bias for c in self.cross])

    def _deep(self, data: Dict[str, Tensor]):
        return self.mlp(self._cross(data))

    def forward(self, data: Dict[str, Tensor]):
        h = self._deep(data)
        return dense_ops.head(h, self.prediction.weight, self.prediction.bias), self._target(data)

    def fused_bce_loss(self, data: Dict[str, Tensor]):
        """Training loss (BCE with logits, mean): the cross network, the deep MLP, the
        output layer and the loss as one fused tower launch (cross layers as tower
        layers with the x0 * (W x + b) + x epilogue, mrec_tower_args.n_cross), else
        the layered cross network ahead of the tower / the output layer fused into
        the loss."""
        x0 = self._x0(data)
        if dense_ops.tower_supported(x0, self.mlp, self.prediction, cross=list(self.cross)):
            return dense_ops.tower_bce(x0, self.mlp, self.prediction, None, self._target(data),
                                       cross=list(self.cross))
        x = dense_ops.cross_net(x0, [c.weight for c in self.cross], [c.bias for c in self.cross])
        if dense_ops.tower_supported(x, self.mlp, self.prediction):
            return dense_ops.tower_bce(x, self.mlp, self.prediction, None, self._target(data))
        loss, _ = dense_ops.ctr_head_bce(self.mlp(x), self.prediction.weight,
                                         self.prediction.bias, None, self._target(data))
        return loss
