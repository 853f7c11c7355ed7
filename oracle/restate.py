"""The build's CPU restatement of the four CTR forwards on the §8 path, in a chosen
numpy dtype (float64 = the parity oracle, float32 = the reference's own arithmetic
width), for golden fixture G9 ("the build's own
FM/DeepFM/DCNv2/DIN CPU restatement outputs in fp64 and fp32").

TEST INFRASTRUCTURE ONLY (imported by tests/ and tests/golden/make_g9.py).

Every function is the composition of oracle/ref.py's cited pieces, restated with
the dtype kept throughout (ref.py promotes to fp64):
  * FM: first order sum_f w[id_f] + dense . w_d + b (SVDPP.py:60-66) plus
    1/2 sum_d[(sum_f v)^2 - sum_f v^2] (FunkSVD.py:51 generalised, ref.fm2);
  * DeepFM: FM + Linear(MLP(x0)) with x0 = [v_1..v_F | dense] (NCF.py:68-74,
    MLP.py:8-23, Dense.py:12-24);
  * DCN-v2: x_{l+1} = x0 * (W_l x_l + b_l) + x_l, then MLP and Linear (ref.dcn_cross_fwd);
  * DIN: scores MLP_att([q, k, q-k, q*k]) -> Linear, masked softmax over valid
    positions (SASRec.py:26-29, utils.py:5-10), u = sum_j a_j k_j (ref.din_attention_pool).
"""
from __future__ import annotations

import numpy as np


def _lin(x, W, b, dt):
    y = x @ np.asarray(W, dt).T
    return y + np.asarray(b, dt) if b is not None else y


def _mlp(x, layers, dt):
    for W, b in layers:
        x = np.maximum(_lin(x, W, b, dt), dt(0))
    return x


def gather_fields(tables, ids, dt):
    """tables: list of [rows_f, D]; ids [B, F] -> v [B, F, D] (nn.Embedding)."""
    return np.stack([np.asarray(t, dt)[ids[:, f]] for f, t in enumerate(tables)], 1)


def fm_logits(tables, wtabs, ids, dense, dense_w, bias, dt):
    v = gather_fields(tables, ids, dt)
    s = v.sum(1)
    fm = dt(0.5) * (s * s - (v * v).sum(1)).sum(-1)
    w = np.stack([np.asarray(t, dt)[ids[:, f]] for f, t in enumerate(wtabs)], 1).sum(1)
    return fm + w + np.asarray(dense, dt) @ np.asarray(dense_w, dt) + dt(bias), v


def deepfm_logits(tables, wtabs, ids, dense, dense_w, bias, mlp, out, dt):
    z, v = fm_logits(tables, wtabs, ids, dense, dense_w, bias, dt)
    x0 = np.concatenate([v.reshape(v.shape[0], -1), np.asarray(dense, dt)], 1)
    return z + _lin(_mlp(x0, mlp, dt), out[0], out[1], dt)[:, 0]


def dcnv2_logits(tables, ids, dense, cross, mlp, out, dt):
    v = gather_fields(tables, ids, dt)
    x0 = np.concatenate([v.reshape(v.shape[0], -1), np.asarray(dense, dt)], 1)
    x = x0
    for W, b in cross:
        x = x0 * _lin(x, W, b, dt) + x
    return _lin(_mlp(x, mlp, dt), out[0], out[1], dt)[:, 0]


def din_pool(q, k, valid, att, att_out, dt):
    q, k = np.asarray(q, dt), np.asarray(k, dt)
    B, L, E = k.shape
    qb = np.broadcast_to(q[:, None, :], k.shape)
    feat = np.concatenate([qb, k, qb - k, qb * k], -1).reshape(B * L, 4 * E)
    s = _lin(_mlp(feat, att, dt), att_out[0], att_out[1], dt).reshape(B, L)
    sm = np.where(np.asarray(valid).astype(bool), s, dt(-np.inf))
    sm = sm - sm.max(-1, keepdims=True)
    e = np.exp(sm)
    a = e / e.sum(-1, keepdims=True)
    return (a[..., None] * k).sum(1), s


def bce_mean(z, y, dt):
    z, y = np.asarray(z, dt), np.asarray(y, dt)
    return (np.maximum(z, dt(0)) - z * y + np.log1p(np.exp(-np.abs(z)))).mean()
