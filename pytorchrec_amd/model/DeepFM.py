"""FM / DeepFM — CTR models on the MI355X hot path.

Neither exists in the reference.  They are built from the
reference's primitives and plug-in contract:
  * tables = ``nn.Embedding`` semantics (FunkSVD.py:39-41) packed in one
    ``EmbeddingBank`` with the first-order weight as an extra column
    (first-order = ``Embedding(rows, 1)`` biases + global bias, SVDPP.py:40-42);
  * FM 2nd order generalises FunkSVD's dot product (FunkSVD.py:51);
  * the deep part is the reference ``MLP`` over the embedding concat (NCF.py:62-74)
    followed by ``Linear(last, 1)``;
  * ``forward(data) -> (prediction, target)`` with target = label.float()
    (FunkSVD.py:53-55).

logit = global_bias + dense . w_dense + sum_f w_f[id_f] + FM2(v) [+ deep(x0)]
with x0 = [v_0 .. v_{F-1} | dense] (26*16 + 13 = 429 wide at Criteo shape).

On a GPU the whole input stage is ONE kernel (``mrec_interact_fwd``) and the
embedding backward is the sorted-segment kernel pair with the SGD update fused.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import torch
from torch import Tensor
from torch.nn import Linear, Parameter

from pytorchrec_amd import dense as dense_ops
from pytorchrec_amd.embedding import interact
from pytorchrec_amd.sharding import make_bank
from pytorchrec_amd.feature_column import CategoricalColumn, NumericColumn
from pytorchrec_amd.model.IModel import IModel
from pytorchrec_amd.model.layer.MLP import MLP
from pytorchrec_amd.utils.argument import ArgumentDescription


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _parse_layers(layers) -> List[int]:
    if isinstance(layers, str):
        return [int(x) for x in layers.replace("[", "").replace("]", "").split(",") if x.strip()]
    return [int(x) for x in layers]


class _CTRBase(IModel):
    """Shared column handling for the CTR models."""

    def _setup_columns(self, sparse_columns, dense_columns, label_column, emb_size, emb_dtype,
                       device):
        self.sparse_columns: List[CategoricalColumn] = list(sparse_columns)
        self.dense_columns: List[NumericColumn] = list(dense_columns or [])
        self.label_column = label_column
        self.emb_size = int(emb_size)
        self.emb_dtype = emb_dtype
        self.build_device = torch.device(device) if device is not None else None

    def _ids(self, data: Dict[str, Tensor]):
        return [c.get_feature_ids(data) for c in self.sparse_columns]

    def _dense(self, data: Dict[str, Tensor]) -> Optional[Tensor]:
        if not self.dense_columns:
            return None
        if "__dense__" in data:  # pre-stacked [B, n_dense] (columnar loaders, bench)
            return data["__dense__"]
        return torch.stack([c.get_feature_data(data) for c in self.dense_columns], dim=1)

    def _target(self, data: Dict[str, Tensor]):
        if self.label_column is None:
            return None
        t = data.get(self.label_column.feature_name)
        return None if t is None else t.float()

    def _x0_dtype(self):
        return torch.bfloat16 if self._on_gpu() else torch.float32

    def _on_gpu(self) -> bool:
        return self.embeddings.weight.is_cuda


class FM(_CTRBase):
    """Factorization Machine: bias + linear + pairwise interactions (config C1)."""

    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return [ArgumentDescription(name="emb_size", type_=int, help_info="embedding dim",
                                    default_value=16, lower_closed_bound=1)]

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        super().check_argument_values(arguments)

    def __init__(self, sparse_columns: Sequence[CategoricalColumn], label_column=None,
                 emb_size: int = 16, dense_columns: Optional[Sequence[NumericColumn]] = None,
                 emb_dtype: torch.dtype = torch.float32, device=None, **kwargs):
        self._setup_columns(sparse_columns, dense_columns, label_column, emb_size, emb_dtype,
                            device)
        super().__init__(**kwargs)

    def _init_weights(self):
        self.embeddings = make_bank([c.category_num for c in self.sparse_columns],
                                        self.emb_size, with_first_order=True,
                                        dtype=self.emb_dtype, device=self.build_device)
        n = len(self.dense_columns)
        self.dense_weight = Parameter(torch.randn(n, device=self.build_device) * 0.01) if n else None
        self.global_bias = Parameter(torch.zeros(1, device=self.build_device))

    def forward(self, data: Dict[str, Tensor]):
        logit = interact(self.embeddings, self._ids(data), self._dense(data), self.dense_weight,
                         self.global_bias, fm2=True, first_order=True)
        return logit, self._target(data)


class DeepFM(_CTRBase):
    """DeepFM: FM (first + second order) and an MLP over the shared embeddings."""

    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return [
            ArgumentDescription(name="emb_size", type_=int, help_info="embedding dim",
                                default_value=16, lower_closed_bound=1),
            ArgumentDescription(name="layers", type_=str, help_info="MLP widths, e.g. 400,400,400",
                                default_value="400,400,400"),
            ArgumentDescription(name="dropout", type_=float, help_info="MLP dropout",
                                default_value=0.0, lower_closed_bound=0.0, upper_open_bound=1.0),
        ]

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        super().check_argument_values(arguments)

    def __init__(self, sparse_columns: Sequence[CategoricalColumn],
                 dense_columns: Optional[Sequence[NumericColumn]] = None, label_column=None,
                 emb_size: int = 16, layers=(400, 400, 400), dropout: float = 0.0,
                 emb_dtype: torch.dtype = torch.float32, device=None, **kwargs):
        self._setup_columns(sparse_columns, dense_columns, label_column, emb_size, emb_dtype,
                            device)
        self.layers = _parse_layers(layers)
        self.dropout = float(dropout)
        super().__init__(**kwargs)

    def _init_weights(self):
        dev = self.build_device
        F, D, n = len(self.sparse_columns), self.emb_size, len(self.dense_columns)
        self.embeddings = make_bank([c.category_num for c in self.sparse_columns], D,
                                        with_first_order=True, dtype=self.emb_dtype, device=dev)
        self.dense_weight = Parameter(torch.randn(n, device=dev) * 0.01) if n else None
        self.global_bias = Parameter(torch.zeros(1, device=dev))
        self.deep_in = F * D + n
        self.x0_cols = _round_up(self.deep_in, 8)  # 16-byte aligned rows; pad is zero
        self.mlp = MLP(self.deep_in, self.layers, "relu", self.dropout)
        self.prediction = Linear(self.layers[-1], 1)
        if dev is not None:
            self.mlp.to(dev)
            self.prediction.to(dev)

    def _deep(self, data: Dict[str, Tensor], dense, with_linear: bool):
        lin = (self.dense_weight, self.global_bias) if with_linear else (None, None)
        x0, logit = interact(self.embeddings, self._ids(data), dense, *lin, fm2=True,
                             first_order=True, x0_cols=self.x0_cols, x0_dtype=self._x0_dtype())
        return self.mlp(x0), logit

    def forward(self, data: Dict[str, Tensor]):
        h, logit = self._deep(data, self._dense(data), True)
        prediction = dense_ops.head(h, self.prediction.weight, self.prediction.bias, base=logit)
        return prediction, self._target(data)

    def fused_bce_loss(self, data: Dict[str, Tensor]):
        """Training loss (BCE with logits, mean): the output layer, the dense
        first-order term + global bias and the loss in one kernel (same sum as
        ``forward`` + the loss, in a different fp32 order)."""
        dense = self._dense(data)
        x0, logit = interact(self.embeddings, self._ids(data), dense, None, None, fm2=True,
                             first_order=True, x0_cols=self.x0_cols, x0_dtype=self._x0_dtype())
        if dense_ops.tower_supported(x0, self.mlp, self.prediction, dense):
            # MLP + output layer + loss and the MLP's input gradients: one launch
            return dense_ops.tower_bce(x0, self.mlp, self.prediction, logit, self._target(data),
                                       xs=dense, ws=self.dense_weight, b2=self.global_bias)
        loss, _ = dense_ops.ctr_head_bce(self.mlp(x0), self.prediction.weight, self.prediction.bias,
                                         logit, self._target(data), xs=dense, ws=self.dense_weight,
                                         b2=self.global_bias)
        return loss
