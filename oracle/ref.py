"""numpy restatement of the hot-path algorithms (TEST INFRASTRUCTURE ONLY).

Every function names the reference code (``/root/reference``) whose behaviour it
restates.  Floating-point functions compute in float64 on whatever inputs they
are given (the GPU parity tests hand them the *same* bf16/fp32 values the kernels
read, upcast), so they are an order-independent ground truth; integer/index
functions are exact.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------
# bf16 helpers (storage format of the MI355X tables; no reference counterpart —
# the reference is fp32 only, IModel.py:61-68 initialises fp32 weights)
# ----------------------------------------------------------------------------


def f32_to_bf16_bits(x) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16, returned as uint16 bit patterns.

    NaN stays NaN (quiet bit forced), matching ``v_cvt_pk_bf16_f32``.
    """
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = x.view(np.uint32).astype(np.uint64)
    rounded = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32)
    nan = np.isnan(x)
    rounded = np.where(nan, ((u >> 16) | 0x40).astype(np.uint32), rounded)
    return rounded.astype(np.uint16)


def bf16_bits_to_f32(b) -> np.ndarray:
    b = np.asarray(b, dtype=np.uint16)
    return (b.astype(np.uint32) << 16).view(np.float32)


def bf16_round(x) -> np.ndarray:
    """fp32 value after a round trip through bf16 (RNE)."""
    return bf16_bits_to_f32(f32_to_bf16_bits(x))


def bf16_ulp(x) -> np.ndarray:
    """Spacing of bf16 numbers at |x| (for 1-ulp tolerance checks)."""
    x = np.abs(np.asarray(x, dtype=np.float64))
    x = np.maximum(x, np.finfo(np.float32).tiny)
    e = np.floor(np.log2(x))
    return np.exp2(e - 7)


# ----------------------------------------------------------------------------
# Feature columns
# ----------------------------------------------------------------------------


def identity_ids(raw) -> np.ndarray:
    """``CategoricalColumnWithIdentity.get_feature_data`` = column cast to int64
    (torchrec/feature_column/CategoricalColumnWithIdentity.py:20-22)."""
    return np.asarray(raw).astype(np.int64)


def crossed_coefficients(category_nums) -> list:
    """Mixed-radix coefficients, last column fastest
    (torchrec/feature_column/CrossedColumn.py:14-22)."""
    coeff = [1] * len(category_nums)
    for i in range(len(category_nums) - 1, 0, -1):
        coeff[i - 1] = coeff[i] * int(category_nums[i])
    return coeff


def crossed_ids(columns_ids, category_nums) -> np.ndarray:
    """``CrossedColumn.get_feature_data``: sum_i coeff_i * id_i, int64, no
    hashing and no overflow guard (CrossedColumn.py:24-27)."""
    coeff = crossed_coefficients(category_nums)
    out = np.zeros(np.asarray(columns_ids[0]).shape, dtype=np.int64)
    for c, ids in zip(coeff, columns_ids):
        out = out + np.int64(c) * np.asarray(ids).astype(np.int64)
    return out


def numeric_normalize(x, mode: str, min_v=0.0, max_v=1.0, mean_v=0.0, std_v=1.0):
    """``NumericColumn.get_feature_data`` (NumericColumn.py:25-34), computed in
    fp32 exactly as torch does: ``(x.float() - a) / b`` with python-float
    scalars promoted to fp32."""
    x = np.asarray(x).astype(np.float32)
    if mode == "nop":
        return x
    if mode == "max_min":
        return ((x - np.float32(min_v)) / np.float32(max_v - min_v)).astype(np.float32)
    if mode == "z_score":
        return ((x - np.float32(mean_v)) / np.float32(std_v)).astype(np.float32)
    raise ValueError(mode)


# ----------------------------------------------------------------------------
# Embedding gather / scatter-add
# ----------------------------------------------------------------------------


def gather(table, ids) -> np.ndarray:
    """``nn.Embedding`` forward: ``out[..., :] = table[ids[...], :]`` as a bit copy
    (built in FunkSVD.py:39-41, used at FunkSVD.py:47-48).  Out-of-range or
    negative ids raise ``IndexError`` as torch does (no ``padding_idx``)."""
    table = np.asarray(table)
    ids = np.asarray(ids).astype(np.int64)
    if ids.size and (ids.min() < 0 or ids.max() >= table.shape[0]):
        raise IndexError("index out of range in self")
    return table[ids]


def multi_table_gather(tables, ids_bf) -> np.ndarray:
    """F independent ``nn.Embedding`` lookups stacked as [B, F, D]; field f reads
    table f (the DeepFM/DCN input of SURVEY.md §8(a) A4)."""
    ids_bf = np.asarray(ids_bf)
    return np.stack([gather(tables[f], ids_bf[:, f]) for f in range(len(tables))], axis=1)


def dense_grad(rows: int, ids, dy) -> np.ndarray:
    """``aten::embedding_dense_backward`` as autograd runs it for ``nn.Embedding``
    (SURVEY.md §8(a) A5): a dense [rows, D] gradient, duplicates summed, row 0
    an ordinary row.  Summed in fp64 in ascending lookup order."""
    ids = np.asarray(ids).reshape(-1).astype(np.int64)
    dy = np.asarray(dy, dtype=np.float64).reshape(ids.shape[0], -1)
    g = np.zeros((rows, dy.shape[1]), dtype=np.float64)
    np.add.at(g, ids, dy)
    return g


def unique_rows_sorted(ids):
    """The row-sparse form of ``dense_grad``: ascending unique rows and, per row,
    the ascending list of lookup positions that hit it.  (The deterministic
    segment order the HIP backward kernel reproduces.)"""
    ids = np.asarray(ids).reshape(-1).astype(np.int64)
    order = np.lexsort((np.arange(ids.shape[0]), ids))
    sorted_ids = ids[order]
    uniq, starts = np.unique(sorted_ids, return_index=True)
    return uniq, order, starts


def sgd_rows(table, ids, dy, lr):
    """Dense SGD (torch.optim.SGD, no momentum / weight decay;
    torchrec/optim/optimizers.py:7-11) applied through ``dense_grad``: only rows
    with a non-zero gradient move, so the row-sparse update is identical."""
    t = np.asarray(table, dtype=np.float64).copy()
    g = dense_grad(t.shape[0], ids, dy)
    return t - lr * g


# ----------------------------------------------------------------------------
# Interactions
# ----------------------------------------------------------------------------


def fm2(v) -> np.ndarray:
    """FM second-order term 1/2 * sum_d[(sum_f v_fd)^2 - sum_f v_fd^2], [B,F,D]->[B].
    The reference's 2-field form is FunkSVD's ``(u*i).sum(-1)`` (FunkSVD.py:51):
    for F=2 the identity gives exactly u.i."""
    v = np.asarray(v, dtype=np.float64)
    s = v.sum(axis=1)
    return 0.5 * (s * s - (v * v).sum(axis=1)).sum(axis=-1)


def fm2_pairwise(v) -> np.ndarray:
    """Same quantity as the explicit pair sum sum_{i<j} <v_i, v_j> (definition)."""
    v = np.asarray(v, dtype=np.float64)
    F = v.shape[1]
    out = np.zeros(v.shape[0])
    for i in range(F):
        for j in range(i + 1, F):
            out += (v[:, i] * v[:, j]).sum(-1)
    return out


def fm2_bwd(v, dy) -> np.ndarray:
    """d fm2 / d v_fd = dy * (S_d - v_fd) with S = sum_f v."""
    v = np.asarray(v, dtype=np.float64)
    dy = np.asarray(dy, dtype=np.float64)
    s = v.sum(axis=1, keepdims=True)
    return dy[:, None, None] * (s - v)


def fm2_magnitude(v) -> np.ndarray:
    """Magnitude-aware denominator for FM parity (SURVEY.md §7 hard part 3):
    1/2 * sum_d (sum_f |v|)^2 bounds every term of the sum-square formula."""
    a = np.abs(np.asarray(v, dtype=np.float64))
    return 0.5 * (a.sum(axis=1) ** 2).sum(axis=-1)


def first_order(w_gathered, dense=None, dense_w=None, bias=0.0) -> np.ndarray:
    """Linear part: sum_f w[id_f] (+ dense . w_dense) + global bias.  Reference
    form: ``u_bias``/``i_bias`` = ``Embedding(rows, 1)`` plus ``global_bias``
    (SVDPP.py:40-42, 60-66)."""
    out = np.asarray(w_gathered, dtype=np.float64).sum(axis=1) + float(bias)
    if dense is not None:
        out = out + np.asarray(dense, np.float64) @ np.asarray(dense_w, np.float64)
    return out


def svdpp_predict(u_tab, i_tab, imp_tab, ub_tab, ib_tab, gbias, u_ids, i_ids, his):
    """SVD++ prediction with masked sum / sqrt(len) history pooling
    (SVDPP.py:44-66, single-item branch)."""
    his = np.asarray(his)
    valid = (his > 0).astype(np.float64)
    hv = gather(imp_tab, his).astype(np.float64)
    imp = (hv * valid[..., None]).sum(axis=1) / np.sqrt(valid.sum(-1))[:, None]
    u = gather(u_tab, u_ids).astype(np.float64)
    i = gather(i_tab, i_ids).astype(np.float64)
    ub = gather(ub_tab, u_ids)[:, 0].astype(np.float64)
    ib = gather(ib_tab, i_ids)[:, 0].astype(np.float64)
    return ((u + imp) * i).sum(-1) + ub + ib + float(gbias)


def valid_his_index(his_ids) -> np.ndarray:
    """``get_valid_his_index``: his_id > 0, position 0 forced valid
    (torchrec/model/utils.py:5-10)."""
    v = (np.asarray(his_ids) > 0).astype(np.uint8)
    v[:, 0] = 1
    return v


def masked_attention(q, k, v, scale=None, attn_mask=None) -> np.ndarray:
    """``scaled_dot_product_attention`` (SASRec.py:14-31): bmm, optional scale,
    subtract the GLOBAL max, mask (mask==1 means *excluded*) with -inf, softmax
    over keys, bmm with v."""
    q = np.asarray(q, np.float64)
    k = np.asarray(k, np.float64)
    v = np.asarray(v, np.float64)
    att = q @ np.swapaxes(k, 1, 2)
    if scale is not None:
        att = att * scale
    att = att - att.max()
    if attn_mask is not None:
        att = np.where(np.asarray(attn_mask).astype(bool), -np.inf, att)
    att = att - att.max(axis=-1, keepdims=True)
    e = np.exp(att)
    p = e / e.sum(-1, keepdims=True)
    return p @ v


# ----------------------------------------------------------------------------
# Dense layers
# ----------------------------------------------------------------------------


def linear(x, W, b=None) -> np.ndarray:
    """``nn.Linear``: x W^T + b, W stored [out, in] (Dense.py:12, NCF.py:51)."""
    y = np.asarray(x, np.float64) @ np.asarray(W, np.float64).T
    if b is not None:
        y = y + np.asarray(b, np.float64)
    return y


def mlp_fwd(x, layers):
    """Reference ``MLP``: per layer Linear -> ReLU -> Dropout (ReLU whatever the
    ``activation`` string, Dense.py:14-24; stacking MLP.py:16-23).  Dropout is
    identity (p=0 / eval).  Returns the list of post-ReLU activations, input
    first."""
    acts = [np.asarray(x, np.float64)]
    for W, b in layers:
        acts.append(np.maximum(linear(acts[-1], W, b), 0.0))
    return acts


def mlp_bwd(acts, layers, dout):
    """Backward of ``mlp_fwd``: returns (dx, [(dW, db), ...])."""
    grads = []
    g = np.asarray(dout, np.float64)
    for li in range(len(layers) - 1, -1, -1):
        W, _ = layers[li]
        g = g * (acts[li + 1] > 0)
        dW = g.T @ acts[li]
        db = g.sum(0)
        grads.append((dW, db))
        g = g @ np.asarray(W, np.float64)
    grads.reverse()
    return g, grads


def dcn_cross_fwd(x0, cross_layers):
    """DCN-v2 full-rank cross stack x_{l+1} = x0 * (W_l x_l + b_l) + x_l (absent
    from the reference; Linear semantics of Dense.py:12).
    Returns (outputs x_0..x_L, pre-products z_0..z_{L-1})."""
    x0 = np.asarray(x0, np.float64)
    xs, zs = [x0], []
    for W, b in cross_layers:
        z = linear(xs[-1], W, b)
        zs.append(z)
        xs.append(x0 * z + xs[-1])
    return xs, zs


def dcn_cross_bwd(xs, zs, cross_layers, dout):
    """Backward of ``dcn_cross_fwd``: returns (dx0_total, [(dW, db), ...])."""
    x0 = xs[0]
    g = np.asarray(dout, np.float64)
    dx0 = np.zeros_like(x0)
    grads = []
    for li in range(len(cross_layers) - 1, -1, -1):
        W, _ = cross_layers[li]
        dz = g * x0
        dx0 += g * zs[li]
        grads.append((dz.T @ xs[li], dz.sum(0)))
        g = g + dz @ np.asarray(W, np.float64)
    grads.reverse()
    return dx0 + g, grads


def din_attention_pool(q, k, valid, att_layers, att_out):
    """DIN target-attention pooling (absent from the reference, SURVEY.md §8(a)
    A11).  Score s_j = MLP_att([q, k_j, q-k_j, q*k_j]) with the reference MLP
    (ReLU layers, Dense.py) followed by a Linear(h, 1); softmax over valid keys
    with invalid keys masked to -inf as ``scaled_dot_product_attention`` does
    (SASRec.py:26-29; validity from ``get_valid_his_index``, utils.py:5-10);
    u = sum_j a_j k_j.

    q [B,E], k [B,L,E], valid [B,L] -> (u [B,E], a [B,L], s [B,L])."""
    q = np.asarray(q, np.float64)
    k = np.asarray(k, np.float64)
    B, L, E = k.shape
    qb = np.broadcast_to(q[:, None, :], k.shape)
    feat = np.concatenate([qb, k, qb - k, qb * k], axis=-1).reshape(B * L, 4 * E)
    acts = mlp_fwd(feat, att_layers)
    Wo, bo = att_out
    s = linear(acts[-1], Wo, bo).reshape(B, L)
    u, a = din_softmax_pool(s, valid, k)
    return u, a, s


def din_softmax_pool(s, valid, k):
    """The pooling half of ``din_attention_pool`` given the scores: masked softmax
    over the valid history positions (invalid -> -inf, then the row max is
    subtracted; SASRec.py:26-29) and u = sum_j a_j k_j.
    s [B,L], valid [B,L], k [B,L,E] -> (u [B,E], a [B,L])."""
    s = np.asarray(s, np.float64)
    k = np.asarray(k, np.float64)
    sm = np.where(np.asarray(valid).astype(bool), s, -np.inf)
    sm = sm - sm.max(-1, keepdims=True)
    e = np.exp(sm)
    a = e / e.sum(-1, keepdims=True)
    return (a[..., None] * k).sum(1), a


def din_softmax_pool_bwd(a, k, du):
    """Backward of ``din_softmax_pool``: with g_j = du . k_j,
    ds_j = a_j (g_j - sum_i a_i g_i) and dk_j = a_j du.  -> (ds [B,L], dk [B,L,E])."""
    a = np.asarray(a, np.float64)
    k = np.asarray(k, np.float64)
    du = np.asarray(du, np.float64)
    g = (k * du[:, None, :]).sum(-1)
    ds = a * (g - (a * g).sum(-1, keepdims=True))
    return ds, a[..., None] * du[:, None, :]


# ----------------------------------------------------------------------------
# Loss
# ----------------------------------------------------------------------------


def bce_with_logits(z, y):
    """``torch.nn.BCEWithLogitsLoss`` (mean) and its gradient w.r.t. the logits."""
    z = np.asarray(z, np.float64)
    y = np.asarray(y, np.float64)
    loss = np.mean(np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z))))
    dz = (1.0 / (1.0 + np.exp(-z)) - y) / z.shape[0]
    return loss, dz


# ----------------------------------------------------------------------------
# Optimizers on a dense table: the reference steps every
# row of every nn.Embedding each step (IModel.py:116-125 -> optimizer.step()).
# ----------------------------------------------------------------------------


def adamw_step(p, g, m, v, t, lr, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0,
               correct_bias=True):
    """One step of the reference AdamW (torchrec/optim/AdamW.py:46-59) on dense
    arrays, in place on p, m, v (float64): m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
    p -= lr sqrt(1-b2^t)/(1-b1^t) m / (sqrt(v) + eps); then p -= lr wd p."""
    b1, b2 = betas
    m *= b1
    m += (1.0 - b1) * g
    v *= b2
    v += (1.0 - b2) * g * g
    step = lr
    if correct_bias:
        step = lr * np.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
    p -= step * m / (np.sqrt(v) + eps)
    if weight_decay > 0.0:
        p -= lr * weight_decay * p


def adam_step(p, g, m, v, t, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    """One step of ``torch.optim.Adam`` (the reference's "adam", optimizers.py:9):
    g += wd p (L2); m, v as AdamW; p -= lr/(1-b1^t) m / (sqrt(v)/sqrt(1-b2^t) + eps)."""
    b1, b2 = betas
    g = g + weight_decay * p if weight_decay else g
    m *= b1
    m += (1.0 - b1) * g
    v *= b2
    v += (1.0 - b2) * g * g
    p -= (lr / (1.0 - b1 ** t)) * m / (np.sqrt(v) / np.sqrt(1.0 - b2 ** t) + eps)


def adagrad_step(p, g, s, lr, eps=1e-10):
    """``torch.optim.Adagrad`` (lr_decay 0, weight_decay 0, initial accumulator 0):
    s += g^2; p -= lr g / (sqrt(s) + eps)."""
    s += g * g
    p -= lr * g / (np.sqrt(s) + eps)


def rowwise_adagrad_step(p, g, s, lr, eps=1e-10):
    """Row-wise Adagrad (pytorchrec_amd.optim.RowWiseAdagrad; no reference
    counterpart): s[r] += mean_d g[r, d]^2; p[r] -= lr g[r] / (sqrt(s[r]) + eps).
    p, g [rows, D]; s [rows]."""
    s += (g * g).mean(axis=1)
    p -= lr * g / (np.sqrt(s)[:, None] + eps)
