"""FunkSVD on the hot path — the reference's only registered model
(torchrec/model/FunkSVD.py:11-67), single-item branch: prediction = u . i,
computed by the fused interaction kernel as the 2-field FM."""
from typing import Any, Dict, List

import torch
from torch import Tensor

from pytorchrec_amd.embedding import EmbeddingBank, interact
from pytorchrec_amd.model.IModel import IModel
from pytorchrec_amd.utils.argument import ArgumentDescription


class FunkSVD(IModel):
    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return [ArgumentDescription(name="emb_size", type_=int, help_info="Embedding层维度",
                                    default_value=64, lower_closed_bound=1)]

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        super().check_argument_values(arguments)

    def __init__(self, uid_column, iid_column, label_column, emb_size: int,
                 emb_dtype: torch.dtype = torch.float32, device=None, **kwargs):
        self.uid_column = uid_column
        self.iid_column = iid_column
        self.label_column = label_column
        self.emb_size = emb_size
        self.emb_dtype = emb_dtype
        self.build_device = device
        super().__init__(**kwargs)

    def _init_weights(self):
        self.embeddings = EmbeddingBank([self.uid_column.category_num,
                                         self.iid_column.category_num], self.emb_size,
                                        dtype=self.emb_dtype, device=self.build_device)

    def forward(self, data: Dict[str, Tensor]):
        i_ids = self.iid_column.get_feature_ids(data)
        if i_ids.dim() != 1:
            raise NotImplementedError("sampled (2-D iid) ranking branch is out of scope")
        prediction = interact(self.embeddings, [self.uid_column.get_feature_ids(data), i_ids],
                              fm2=True, first_order=False)
        target = None
        if self.label_column is not None and self.label_column.feature_name in data:
            target = data[self.label_column.feature_name].float()
        return prediction, target
