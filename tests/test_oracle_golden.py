"""Pin the CPU oracle (oracle/ref.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import os
import sys

import numpy as np
import pytest

from conftest import golden
from oracle import ref


def test_g1_gather_fp32_bit_exact():
    g = golden("g1_gather.npz")
    out = ref.gather(g["table"], g["ids"])
    assert out.dtype == np.float32
    assert np.array_equal(out.view(np.uint32), g["out"].view(np.uint32))


def test_g1_gather_bf16_bit_exact():
    g = golden("g1_gather.npz")
    out = ref.gather(g["table_bf16"], g["ids"])
    assert np.array_equal(out, g["out_bf16"])
    # the bf16 table is the RNE rounding of the fp32 one (what the kernels store)
    assert np.array_equal(ref.f32_to_bf16_bits(g["table"]), g["table_bf16"])


def test_g1_gather_oob_raises_index_error():
    g = golden("g1_gather.npz")
    assert bool(g["oob_raises"])
    with pytest.raises(IndexError):
        ref.gather(g["table"], np.array([g["table"].shape[0]]))
    with pytest.raises(IndexError):
        ref.gather(g["table"], np.array([-1]))


def test_g2_dense_grad():
    g = golden("g2_dense_grad.npz")
    got = ref.dense_grad(int(g["rows"]), g["ids"], g["dy"])
    np.testing.assert_allclose(got, g["grad"], rtol=1e-6, atol=1e-6)
    # duplicates accumulate, untouched rows are exactly zero
    untouched = np.setdiff1d(np.arange(int(g["rows"])), g["ids"])
    assert np.all(g["grad"][untouched] == 0)


def test_g3_funksvd_is_two_field_fm():
    g = golden("g3_funksvd.npz")
    v = np.stack([ref.gather(g["u_table"], g["uid"]), ref.gather(g["i_table"], g["iid"])], 1)
    fm = ref.fm2(v)
    np.testing.assert_allclose(fm, g["prediction"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(ref.fm2_pairwise(v), fm, rtol=1e-12, atol=1e-15)
    assert np.array_equal(g["target"], g["label"].astype(np.float32))


def test_g10_funksvd_sgd_step_is_row_sparse_sgd():
    g = golden("g10_funksvd_sgd_step.npz")
    u = g["u_before"].astype(np.float64)
    i = g["i_before"].astype(np.float64)
    uv, iv = u[g["uid"]], i[g["iid"]]
    pred = (uv * iv).sum(-1)
    y = g["label"].astype(np.float64)
    loss = np.mean((pred - y) ** 2)
    np.testing.assert_allclose(loss, float(g["loss"]), rtol=1e-5)
    dpred = 2.0 * (pred - y) / pred.shape[0]
    lr = float(g["lr"])
    u_new = ref.sgd_rows(u, g["uid"], dpred[:, None] * iv, lr)
    i_new = ref.sgd_rows(i, g["iid"], dpred[:, None] * uv, lr)
    np.testing.assert_allclose(u_new, g["u_after"], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(i_new, g["i_after"], rtol=1e-5, atol=1e-8)
    # rows never looked up are bit-identical (row-sparse == dense SGD w/o momentum)
    untouched = np.setdiff1d(np.arange(u.shape[0]), g["uid"])
    assert np.array_equal(g["u_after"][untouched], g["u_before"][untouched])


def test_g4_svdpp_pooling_and_biases():
    g = golden("g4_svdpp.npz")
    got = ref.svdpp_predict(g["u_table"], g["i_table"], g["imp_table"], g["ub_table"],
                            g["ib_table"], g["global_bias"], g["uid"], g["iid"], g["his"])
    np.testing.assert_allclose(got, g["prediction"], rtol=1e-5, atol=1e-7)


def test_g5_sasrec_masked_attention():
    g = golden("g5_sasrec_attn.npz")
    assert np.array_equal(ref.valid_his_index(g["his_ids"]), g["valid"])
    got = ref.masked_attention(g["q"], g["k"], g["k"], scale=float(g["scale"]), attn_mask=g["mask"])
    np.testing.assert_allclose(got, g["context"], rtol=1e-5, atol=1e-6)


def test_g5_din_pooling_reduces_to_sasrec_softmax():
    """With a score MLP that computes q.k*scale exactly, DIN pooling == SASRec
    masked attention: pins the mask/softmax/pooling semantics of A11."""
    g = golden("g5_sasrec_attn.npz")
    q = g["q"][:, 0, :].astype(np.float64)
    k = g["k"].astype(np.float64)
    E = q.shape[1]
    # feature = [q, k, q-k, q*k]; a Linear picking sum(q*k)*scale, then the
    # reference MLP with zero layers, then identity output.
    Wo = np.zeros((1, 4 * E))
    Wo[0, 3 * E:] = float(g["scale"])
    u, a, s = ref.din_attention_pool(q, k, g["valid"], [], (Wo, np.zeros(1)))
    np.testing.assert_allclose(u, g["context"][:, 0, :], rtol=1e-5, atol=1e-6)


def test_g6_reference_mlp_fwd_bwd():
    g = golden("g6_mlp.npz")
    n = int(g["n_layers"])
    layers = [(g[f"W{i}"], g[f"b{i}"]) for i in range(n)]
    acts = ref.mlp_fwd(g["x"], layers)
    np.testing.assert_allclose(acts[-1], g["y"], rtol=1e-5, atol=1e-6)
    dx, grads = ref.mlp_bwd(acts, layers, g["dout"])
    np.testing.assert_allclose(dx, g["dx"], rtol=1e-5, atol=1e-6)
    for i, (dW, db) in enumerate(grads):
        # fp32 golden vs fp64 oracle: the sums over the batch cancel, so the
        # tolerance is scaled by the tensor's magnitude (SURVEY.md §7 part 3)
        for got, want in ((dW, g[f"dW{i}"]), (db, g[f"db{i}"])):
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6 * np.abs(want).max())


def test_g7_ncf_concat_mlp_linear():
    g = golden("g7_ncf.npz")
    sample_n = g["iid"].shape[1]
    u = np.repeat(g["uid"][:, None], sample_n, 1).reshape(-1)
    i = g["iid"].reshape(-1)
    mf = ref.gather(g["mf_u"], u).astype(np.float64) * ref.gather(g["mf_i"], i)
    x = np.concatenate([ref.gather(g["mlp_u"], u), ref.gather(g["mlp_i"], i)], -1)
    h = ref.mlp_fwd(x, [(g["W0"], g["b0"]), (g["W1"], g["b1"])])[-1]
    pred = ref.linear(np.concatenate([mf, h], -1), g["Wp"]).reshape(-1, sample_n)
    np.testing.assert_allclose(pred, g["prediction"], rtol=1e-5, atol=1e-7)


def test_g8_feature_columns():
    g = golden("g8_columns.npz")
    coeff = ref.crossed_coefficients([7, 5, 3])
    assert coeff == list(g["coefficients"])
    assert np.array_equal(ref.crossed_ids([g["a"], g["b"], g["c"]], [7, 5, 3]), g["crossed"])
    assert int(g["category_num"]) == 105
    assert np.array_equal(ref.numeric_normalize(g["x"], "nop"), g["nop"])
    np.testing.assert_array_equal(ref.numeric_normalize(g["x"], "max_min", -3.0, 7.0), g["max_min"])
    np.testing.assert_array_equal(ref.numeric_normalize(g["x"], "z_score", mean_v=2.0, std_v=2.9),
                                  g["z_score"])


def test_fm2_identity_and_bwd_finite_difference():
    rng = np.random.default_rng(0)
    v = rng.standard_normal((5, 7, 4))
    np.testing.assert_allclose(ref.fm2(v), ref.fm2_pairwise(v), rtol=1e-12)
    dy = rng.standard_normal(5)
    dv = ref.fm2_bwd(v, dy)
    eps = 1e-6
    vp = v.copy()
    vp[2, 3, 1] += eps
    num = ((ref.fm2(vp) - ref.fm2(v)) * dy).sum() / eps
    np.testing.assert_allclose(dv[2, 3, 1], num, rtol=1e-5)


def test_dcn_cross_bwd_finite_difference():
    rng = np.random.default_rng(1)
    d = 6
    layers = [(rng.standard_normal((d, d)) * 0.3, rng.standard_normal(d) * 0.1) for _ in range(3)]
    x0 = rng.standard_normal((4, d))
    dout = rng.standard_normal((4, d))
    xs, zs = ref.dcn_cross_fwd(x0, layers)
    dx0, grads = ref.dcn_cross_bwd(xs, zs, layers, dout)
    eps = 1e-6
    xp = x0.copy()
    xp[1, 2] += eps
    num = ((ref.dcn_cross_fwd(xp, layers)[0][-1] - xs[-1]) * dout).sum() / eps
    np.testing.assert_allclose(dx0[1, 2], num, rtol=1e-5)
    W0p = [(layers[0][0].copy(), layers[0][1])] + layers[1:]
    W0p[0][0][3, 4] += eps
    num = ((ref.dcn_cross_fwd(x0, W0p)[0][-1] - xs[-1]) * dout).sum() / eps
    np.testing.assert_allclose(grads[0][0][3, 4], num, rtol=1e-5)


def test_bf16_rne_matches_torch():
    import torch
    x = np.random.default_rng(2).standard_normal(4096).astype(np.float32) * 10
    x[:4] = [0.0, -0.0, np.inf, -np.inf]
    t = torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(ref.f32_to_bf16_bits(x), t)


# ---- G9: the build's own restatement (oracle/restate.py), fp64 and fp32 ----------

def _g9():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_g9
    return make_g9


def test_g9_restatement_pinned_fp64_fp32():
    """Recompute every G9 output in both widths: fp64 must reproduce the fixture to
    rounding, fp32 to fp32 reassociation (BLAS blocking may differ by machine)."""
    m, g = _g9(), golden("g9_restatement.npz")
    a = {k: g[k] for k in g.files}
    for name, dt, rtol in (("f64", np.float64, 1e-12), ("f32", np.float32, 2e-5)):
        got = m.small_outputs(a, dt)
        for k, v in got.items():
            want = g[f"{k}_{name}"]
            np.testing.assert_allclose(np.asarray(v, np.float64), want, rtol=rtol,
                                       atol=rtol * np.abs(want).max(), err_msg=f"{k}_{name}")
    # fp32 vs fp64: what the reference's own fp32 arithmetic costs on this path
    for k in ("fm", "deepfm", "dcnv2", "din_u"):
        w = g[f"{k}_f64"]
        assert np.max(np.abs(g[f"{k}_f32"] - w)) <= 1e-5 * np.abs(w).max(), k


def test_g9_restatement_agrees_with_cited_pieces():
    """restate.py's fp64 path == the composition of ref.py's cited functions."""
    g = golden("g9_restatement.npz")
    tabs, ids = list(g["tables"]), g["ids"]
    v = np.stack([ref.gather(t, ids[:, f]) for f, t in enumerate(tabs)], 1)
    wg = np.stack([g["wtabs"][f][ids[:, f]] for f in range(len(tabs))], 1)
    fm = ref.fm2(v) + ref.first_order(wg, g["dense"], g["dense_w"], float(g["bias"]))
    np.testing.assert_allclose(fm, g["fm_f64"], rtol=1e-12, atol=1e-14)
    mlp = [(g["mlp_W0"], g["mlp_b0"]), (g["mlp_W1"], g["mlp_b1"])]
    x0 = np.concatenate([v.reshape(v.shape[0], -1), g["dense"]], 1)
    deep = ref.linear(ref.mlp_fwd(x0, mlp)[-1], g["out_W"], g["out_b"])[:, 0]
    np.testing.assert_allclose(fm + deep, g["deepfm_f64"], rtol=1e-12, atol=1e-14)
    xs, _ = ref.dcn_cross_fwd(x0, [(g[f"cross_W{i}"], g[f"cross_b{i}"]) for i in range(3)])
    dcn = ref.linear(ref.mlp_fwd(xs[-1], mlp)[-1], g["out_W"], g["out_b"])[:, 0]
    np.testing.assert_allclose(dcn, g["dcnv2_f64"], rtol=1e-12, atol=1e-14)
    u, _, s = ref.din_attention_pool(g["din_q"], g["din_k"], g["din_valid"],
                                     [(g["din_att_W0"], g["din_att_b0"])],
                                     (g["din_out_W"], g["din_out_b"]))
    np.testing.assert_allclose(u, g["din_u_f64"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(s, g["din_s_f64"], rtol=1e-12, atol=1e-14)
    z, dz = ref.bce_with_logits(g["deepfm_f64"], g["label"])
    np.testing.assert_allclose(z, float(g["deepfm_loss_f64"]), rtol=1e-12)


def test_g9_full_size_c2_hash_and_checksum():
    """The B = 4096 C2 case: seeded inputs hash exactly; the fp64 FM logits'
    checksum (sum, sum |z|, first 32) is reproduced."""
    m, g = _g9(), golden("g9_restatement.npz")
    tables, wtabs, ids, dense, dense_w = m.c2_inputs()
    assert m.c2_hash(tables, wtabs, ids, dense, dense_w) == str(g["c2_sha256"])
    from oracle import restate
    z, _ = restate.fm_logits(list(tables), list(wtabs), ids, dense, dense_w, 0.0, np.float64)
    sums, head = m.c2_checksum(z)
    np.testing.assert_allclose(sums, g["c2_fm_sums"], rtol=1e-10)
    np.testing.assert_allclose(head, g["c2_fm_head"], rtol=1e-12)


def test_refdin_model_agrees_with_numpy_oracle_and_bf16_emulation_is_close():
    """oracle.models.RefDIN (the C4 step oracle, fp64) against the numpy
    restatement ``ref.din_attention_pool`` (pinned to the reference's masked
    softmax by G5 above) and the reference MLP (``ref.mlp_fwd``, pinned by G6): the
    same logits on a small seeded batch with ragged histories, PAD positions
    included.  Its ``bf16_points`` twin stays within a few percent of it (that
    distance sizes the C4 GPU test's bar)."""
    import torch
    from oracle.models import RefDIN, din_batch
    r = RefDIN(501, 37, 16, (80, 40), (200, 80), dtype=torch.float64)
    with torch.no_grad():
        for p in list(r.att_mlp.parameters()) + list(r.att_out.parameters()):
            p.mul_(40.0)
        for t in (r.item, r.cate):
            t.weight.mul_(10.0)
    iid, cid, his, hcat, _ = din_batch(501, 37, 64, 50, seed=4)
    assert (his == 0).any() and (his[:, 0] > 0).all()
    with torch.no_grad():
        got = r(iid, cid, his, hcat).numpy()
        q = torch.cat([r.item(iid), r.cate(cid)], -1).numpy()
        k = torch.cat([r.item(his), r.cate(hcat)], -1).numpy()
        lin = lambda ms: [(m.weight.numpy(), m.bias.numpy()) for m in ms  # noqa: E731
                          if isinstance(m, torch.nn.Linear)]
        u, a, s = ref.din_attention_pool(q, k, ref.valid_his_index(his.numpy()), lin(r.att_mlp),
                                         (r.att_out.weight.numpy(), r.att_out.bias.numpy()))
        assert np.all(a[ref.valid_his_index(his.numpy()) == 0] == 0)
        h = ref.mlp_fwd(np.concatenate([q, u], 1), lin(r.mlp))[-1]
        want = ref.linear(h, r.out.weight.numpy(), r.out.bias.numpy())[:, 0]
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    e = RefDIN(501, 37, 16, (80, 40), (200, 80), dtype=torch.float32, bf16_points=True)
    e.load_state_dict({k_: v.float() for k_, v in r.state_dict().items()})
    with torch.no_grad():
        emu = e(iid, cid, his, hcat).double().numpy()
    assert np.abs(emu - got).max() <= 0.05 * np.abs(got).max()
