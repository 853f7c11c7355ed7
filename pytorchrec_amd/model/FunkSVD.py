"""FunkSVD on the hot path — the reference's only registered model
(torchrec/model/FunkSVD.py:11-67).

Both branches of the reference ``forward`` run on the fused interaction kernel as
the 2-field FM (u . i == FM over {uid, iid}):
  * single item, ``iid`` [B]: prediction [B], target = label.float()
    (FunkSVD.py:50-55);
  * sampled, ``iid`` [B, N] (the reference's ranking / evaluation branch,
    FunkSVD.py:56-65): prediction [B, N] = u_b . i_{b,n} (the uid of sample b is
    repeated for its N candidates), target [B, N] float32 with column 0 = 1.

Checkpoint compatibility: the two tables live in ONE ``EmbeddingBank`` (one
gather launch for both), but ``state_dict`` / ``load_state_dict`` speak the
reference's keys ``u_embeddings.weight`` [users, emb] and
``i_embeddings.weight`` [items, emb] (FunkSVD.py:39-41), so a reference
checkpoint loads and a checkpoint saved here loads into the reference.
Initialisation consumes the CPU RNG exactly as the reference does (two
``nn.Embedding`` constructions, then ``IModel._reset_weights`` per table), so
the same ``random_seed`` gives bit-identical tables (pinned by golden G10).
"""
from typing import Any, Dict, List

import torch
from torch import Tensor

from pytorchrec_amd.embedding import EmbeddingBank, interact
from pytorchrec_amd.model.IModel import IModel
from pytorchrec_amd.utils.argument import ArgumentDescription

_U_KEY, _I_KEY, _BANK_KEY = "u_embeddings.weight", "i_embeddings.weight", "embeddings.weight"


def _state_dict_hook(module, state_dict, prefix, local_metadata):
    """embeddings.weight -> the reference's u_embeddings.weight / i_embeddings.weight."""
    w = state_dict.pop(prefix + _BANK_KEY, None)
    if w is None:
        return state_dict
    nu, D = module.uid_column.category_num, module.emb_size
    state_dict[prefix + _U_KEY] = w[:nu, :D].clone()
    state_dict[prefix + _I_KEY] = w[nu:, :D].clone()
    return state_dict


def _load_pre_hook(module, state_dict, prefix, local_metadata, strict, missing_keys,
                   unexpected_keys, error_msgs):
    """The reference keys (or the packed bank key) -> the packed bank weight."""
    ku, ki = prefix + _U_KEY, prefix + _I_KEY
    if ku not in state_dict and ki not in state_dict:
        return
    bank = module.embeddings
    nu, D = module.uid_column.category_num, module.emb_size
    w = bank.weight.detach().clone()
    for key, sl in ((ku, slice(0, nu)), (ki, slice(nu, bank.total_rows))):
        t = state_dict.pop(key, None)
        if t is None:
            if strict:
                missing_keys.append(key)
            continue
        want = (sl.stop - sl.start, D)
        if tuple(t.shape) != want:
            error_msgs.append(f"size mismatch for {key}: copying a param with shape "
                              f"{tuple(t.shape)}, the shape in current model is {want}.")
            continue
        w[sl, :D] = t.to(device=w.device, dtype=w.dtype)
    state_dict[prefix + _BANK_KEY] = w


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
        self._register_state_dict_hook(_state_dict_hook)
        self._register_load_state_dict_pre_hook(_load_pre_hook, with_module=True)

    def _init_weights(self):
        self.embeddings = EmbeddingBank([self.uid_column.category_num,
                                         self.iid_column.category_num], self.emb_size,
                                        dtype=self.emb_dtype, device=self.build_device)
        # nn.Embedding's constructor draws N(0, 1) for each table (u, then i): keep
        # the RNG stream where the reference has it
        self._init_tables(1.0)

    def _init_tables(self, std: float):
        """normal(0, std) per table in the reference's order (u, then i), drawn on the
        CPU default generator like the reference's CPU-built model, then copied."""
        bank = self.embeddings
        with torch.no_grad():
            if bank.row_stride != self.emb_size:
                bank.weight.zero_()  # row padding stays zero
            for f, n in enumerate(bank.category_nums):
                t = torch.empty(n, self.emb_size)
                torch.nn.init.normal_(t, mean=0.0, std=std)
                bank.table(f).copy_(t.to(bank.weight.dtype))

    def _reset_weights(self):
        # IModel._reset_weights_fn visits u_embeddings then i_embeddings
        # (IModel.py:61-68): normal(0, 0.01) each
        self._init_tables(0.01)

    def forward(self, data: Dict[str, Tensor]):
        u_ids = self.uid_column.get_feature_ids(data)
        i_ids = self.iid_column.get_feature_ids(data)
        if i_ids.dim() == 1:
            prediction = interact(self.embeddings, [u_ids, i_ids], fm2=True, first_order=False)
            target = None
            if self.label_column is not None and self.label_column.feature_name in data:
                target = data[self.label_column.feature_name].float()
            return prediction, target
        # sampled branch (FunkSVD.py:56-65): every (sample, candidate) pair is one
        # 2-field interaction row
        B, N = i_ids.shape
        uu = u_ids.reshape(B, 1).expand(B, N).reshape(-1).contiguous()
        prediction = interact(self.embeddings, [uu, i_ids.reshape(-1).contiguous()], fm2=True,
                              first_order=False).reshape(B, N)
        target = torch.zeros_like(prediction, dtype=torch.float32)
        target[:, 0] = 1
        return prediction, target
