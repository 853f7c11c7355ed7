"""DIN — Deep Interest Network with target-attention pooling (config C4).

Absent from the reference; built from its idioms:
  * padded history ``pos_his`` [B, L] with 0 = PAD, tail-padded
    (interaction_history_list.py:17-29); validity = his_id > 0 with position 0
    forced valid (``get_valid_his_index``, torchrec/model/utils.py:5-10);
  * masked softmax with -inf on invalid keys (SASRec.py:26-29) — this build uses
    the softmax variant of DIN (the official-code form) and documents it;
  * item and category tables shared between the target and the history;
  * attention unit = reference ``MLP`` over [q, k, q-k, q*k] + ``Linear(h, 1)``;
    top = ``MLP`` over [q, u] + ``Linear(last, 1)``.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import torch
from torch import Tensor
from torch.nn import Linear

from pytorchrec_amd import dense as dense_ops
from pytorchrec_amd.embedding import gather
from pytorchrec_amd.sharding import make_bank
from pytorchrec_amd.feature_column import CategoricalColumn
from pytorchrec_amd.model.DeepFM import _parse_layers
from pytorchrec_amd.model.IModel import IModel
from pytorchrec_amd.model.layer.MLP import MLP
from pytorchrec_amd.utils.argument import ArgumentDescription


def din_lookup_ids(iid: Tensor, cid: Tensor, his: Tensor, hcat: Tensor, rows=None):
    """[target ids | history ids, invalid positions -1] for the item and category
    tables (int32, one kernel: mrec_din_lookup_ids).  A looked-up id that is negative
    or past int32 becomes INT32_MAX, which the gather's range check reports as
    IndexError (``rows``: the two tables' row counts, all below INT32_MAX)."""
    from pytorchrec_amd import _mrec
    if rows is not None and max(rows) >= 2 ** 31 - 1:
        raise ValueError("DIN padded lookups need tables of fewer than 2^31 - 1 rows")
    B, L = his.shape
    dt = his.dtype
    iid, cid = iid.reshape(-1).to(dt).contiguous(), cid.reshape(-1).to(dt).contiguous()
    hcat = hcat.to(dt)
    if his.stride(1) != 1:
        his = his.contiguous()
    if hcat.stride(1) != 1:
        hcat = hcat.contiguous()
    out_i = torch.empty(B * (L + 1), dtype=torch.int32, device=his.device)
    out_c = torch.empty_like(out_i)
    _mrec.call("mrec_din_lookup_ids", iid.data_ptr(), cid.data_ptr(), his.data_ptr(),
               his.stride(0), hcat.data_ptr(), hcat.stride(0), _mrec.dtype_code(dt), B, L,
               out_i.data_ptr(), out_c.data_ptr(), _mrec.stream_handle())
    return out_i, out_c


def din_id_buffers(his: Tensor):
    """int32 [B (L + 1)] item / category lookup-id buffers for mrec_din_gather."""
    B, L = his.shape
    out_i = torch.empty(B * (L + 1), dtype=torch.int32, device=his.device)
    return [out_i, torch.empty_like(out_i)]


def din_sources(iid: Tensor, cid: Tensor, his: Tensor, hcat: Tensor, rows=None):
    """(iid, cid, his, hcat) of one id dtype, rows contiguous (mrec_din_gather's inputs)."""
    if rows is not None and max(rows) >= 2 ** 31 - 1:
        raise ValueError("DIN padded lookups need tables of fewer than 2^31 - 1 rows")
    dt = his.dtype
    iid, cid = iid.reshape(-1).to(dt).contiguous(), cid.reshape(-1).to(dt).contiguous()
    hcat = hcat.to(dt)
    if his.stride(1) != 1:
        his = his.contiguous()
    if hcat.stride(1) != 1:
        hcat = hcat.contiguous()
    return iid, cid, his, hcat


class DIN(IModel):
    # GPU: masked history positions are padding slots of the lookup (see _top);
    # False keeps the plain [target | history] ids (A/B, parity tests)
    pad_skip = True

    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return [
            ArgumentDescription(name="emb_size", type_=int, help_info="embedding dim",
                                default_value=16, lower_closed_bound=1),
            ArgumentDescription(name="att_layers", type_=str, help_info="attention MLP widths",
                                default_value="80,40"),
            ArgumentDescription(name="layers", type_=str, help_info="top MLP widths",
                                default_value="200,80"),
        ]

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        super().check_argument_values(arguments)

    def __init__(self, iid_column: CategoricalColumn, cid_column: CategoricalColumn,
                 his_column: CategoricalColumn, his_cate_column: CategoricalColumn,
                 label_column=None, emb_size: int = 16, att_layers=(80, 40), layers=(200, 80),
                 dropout: float = 0.0, emb_dtype: torch.dtype = torch.float32, device=None,
                 **kwargs):
        self.iid_column = iid_column
        self.cid_column = cid_column
        self.his_column = his_column
        self.his_cate_column = his_cate_column
        self.label_column = label_column
        self.emb_size = int(emb_size)
        self.att_layers = _parse_layers(att_layers)
        self.layers = _parse_layers(layers)
        self.dropout = float(dropout)
        self.emb_dtype = emb_dtype
        self.build_device = torch.device(device) if device is not None else None
        super().__init__(**kwargs)

    def _init_weights(self):
        dev = self.build_device
        D = self.emb_size
        self.embeddings = make_bank([self.iid_column.category_num,
                                         self.cid_column.category_num], D,
                                        with_first_order=False, dtype=self.emb_dtype, device=dev)
        E = 2 * D
        self.att_mlp = MLP(4 * E, self.att_layers, "relu", 0.0)
        self.att_out = Linear(self.att_layers[-1], 1)
        self.mlp = MLP(2 * E, self.layers, "relu", self.dropout)
        self.prediction = Linear(self.layers[-1], 1)
        if dev is not None:
            for m in (self.att_mlp, self.att_out, self.mlp, self.prediction):
                m.to(dev)

    def _top(self, data: Dict[str, Tensor]):
        bank = self.embeddings
        on_gpu = bank.weight.is_cuda
        act_dtype = torch.bfloat16 if on_gpu else torch.float32
        iid = self.iid_column.get_feature_ids(data)
        cid = self.cid_column.get_feature_ids(data)
        his = self.his_column.get_feature_ids(data)
        hcat = self.his_cate_column.get_feature_ids(data)
        B, L = his.shape
        # target and history rows in ONE lookup per table (one sorted-segment
        # backward, one SGD update per row, as a single nn.Embedding call would do)
        if on_gpu and self.pad_skip:
            # masked history positions (softmax weight 0: an exactly zero gradient)
            # become padding slots (-1): zero rows forward, skipped by the backward, so
            # the PAD row is not a ~B L / 2-lookup hot row of every step's update
            if bank.update == "adam":  # rows are caught up on read: the plain gather
                ids_i, ids_c = din_lookup_ids(iid, cid, his, hcat, bank.category_nums)
                rows = gather(bank, [ids_i, ids_c], out_dtype=act_dtype, pad_negative=True)
            else:  # ids built inside the gather launch (mrec_din_gather)
                rows = gather(bank, din_id_buffers(his), out_dtype=act_dtype, pad_negative=True,
                              din_src=din_sources(iid, cid, his, hcat, bank.category_nums))
            return dense_ops.din_attention_top_rows(rows, B, his, self.att_mlp, self.att_out)
        rows = gather(bank, [torch.cat([iid.reshape(-1), his.reshape(-1).to(iid.dtype)]),
                             torch.cat([cid.reshape(-1), hcat.reshape(-1).to(cid.dtype)])],
                      out_dtype=act_dtype)
        if on_gpu:
            return dense_ops.din_attention_top_rows(rows, B, his, self.att_mlp, self.att_out)
        q, k = rows[:B], rows[B:]
        valid = his > 0
        valid[:, 0] = True
        u = dense_ops.din_attention(q, k.reshape(B, L, -1), valid, self.att_mlp, self.att_out)
        return torch.cat([q.float(), u], dim=-1)

    def forward(self, data: Dict[str, Tensor]):
        h = self.mlp(self._top(data))
        logit = dense_ops.head(h, self.prediction.weight, self.prediction.bias)
        target = None
        if self.label_column is not None and self.label_column.feature_name in data:
            target = data[self.label_column.feature_name].float()
        return logit.reshape(-1).float(), target

    def fused_bce_loss(self, data: Dict[str, Tensor]):
        """Training loss (BCE with logits, mean) with the output layer fused into it."""
        top = self._top(data)
        y = data[self.label_column.feature_name].float()
        if dense_ops.tower_supported(top, self.mlp, self.prediction):
            return dense_ops.tower_bce(top, self.mlp, self.prediction, None, y)
        h = self.mlp(top)
        loss, _ = dense_ops.ctr_head_bce(h, self.prediction.weight, self.prediction.bias, None, y)
        return loss
