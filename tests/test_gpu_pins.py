"""GPU parity pins for the configs and composites the per-kernel tests do not
reach (VERDICT r01 "Next round" item 1):

  * C3 at its own shape: the DCN-v2 cross network at d = 429 (ld 432), 3 layers,
    B = 4096 against ``ref.dcn_cross_fwd/bwd``; a full DCN-v2 train step at the C3
    shape (26 x 38,462 rows, D = 16, 13 dense, deep 400-400) against the oracle's
    reference-path model ``RefDCNv2`` in fp64;
  * C5 indexing: gather and fused SGD on rows whose element offset in the bank
    exceeds 2^31 (byte offset > 2^32), bit-exact / 1-ulp against the oracle;
  * the product ``FunkSVD.train_step`` against golden G10 (produced by the
    reference's own ``IModel.train_step``, fp32, IModel.py:116-125) and its sampled
    branch against G11 (FunkSVD.py:56-65);
  * the DIN masked-softmax pooling kernels in isolation (fp32 arithmetic) against
    ``ref.din_softmax_pool(_bwd)`` at 1e-5.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def _ulp_close(got_bits, want_f64, ulps=1):
    got = ref.bf16_bits_to_f32(got_bits).astype(np.float64)
    return np.abs(got - want_f64) <= ulps * ref.bf16_ulp(want_f64) * 1.0001


# ---------------------------------------------------------------------------
# C3: cross network at d = 429, B = 4096
# ---------------------------------------------------------------------------

def test_c3_cross_net_at_config_shape(gpu):
    """x_{l+1} = x0 * (W_l x_l + b_l) + x_l, l = 0..2, d = 429 (x0 rows padded to 432),
    B = 4096: forward and every gradient against the fp64 oracle on the same
    bf16 x0 / fp32 W.  bf16 activations through 3 layers (each x_l and z_l is
    rounded once) -> 3 % of the tensor's magnitude, and the median element
    within 1 %."""
    from pytorchrec_amd import dense as D
    rng = np.random.default_rng(303)
    M, d, L = 4096, 429, 3
    x0 = torch.from_numpy(rng.standard_normal((M, d)).astype(np.float32)).to(torch.bfloat16)
    W = [torch.from_numpy((rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32))
         for _ in range(L)]
    b = [torch.from_numpy((rng.standard_normal(d) * 0.1).astype(np.float32)) for _ in range(L)]
    Wg = [w.to(gpu).requires_grad_() for w in W]
    bg = [v.to(gpu).requires_grad_() for v in b]
    x0p = torch.zeros(M, D._r8(d), dtype=torch.bfloat16, device=gpu)
    x0p[:, :d] = x0.to(gpu)
    x0g = x0p[:, :d].detach().requires_grad_()
    assert x0g.stride(0) == 432
    x = D.cross_net(x0g, Wg, bg)
    dout = (rng.standard_normal((M, d)) * 0.1).astype(np.float32)
    x.backward(torch.from_numpy(dout).to(gpu).to(x.dtype))
    layers = [(w.numpy(), v.numpy()) for w, v in zip(W, b)]
    xs, zs = ref.dcn_cross_fwd(x0.float().numpy(), layers)
    dx0, grads = ref.dcn_cross_bwd(xs, zs, layers, ref.bf16_round(dout))

    def check(got, want, name):
        got = got.detach().double().cpu().numpy()
        mag = np.abs(want).max()
        err = np.abs(got - want)
        assert err.max() <= 0.03 * mag, (name, err.max() / mag)
        assert np.median(err / (np.abs(want) + 1e-3 * mag)) <= 1e-2, name

    check(x, xs[-1], "x_L")
    check(x0g.grad, dx0, "dx0")
    for i in range(L):
        check(Wg[i].grad, grads[i][0], f"dW{i}")
        check(bg[i].grad, grads[i][1], f"db{i}")


def _dcnv2_pair(gpu, rows, B, scale_cross=8.0, scale_mlp=6.0, emb_dtype=torch.float32):
    import torch.nn as nn
    from oracle.models import RefDCNv2
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DCNv2
    nums = [rows] * 26
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{f + 1}") for f, n in enumerate(nums)]
    dense = [NumericColumn(f"c_n_I{j + 1}") for j in range(13)]
    lab = CategoricalColumnWithIdentity(2, "label")
    m = DCNv2(sparse, dense, lab, emb_size=16, cross_layers=3, layers=(400, 400),
              emb_dtype=emb_dtype, device=gpu, random_seed=2020)
    m.embeddings.stochastic_rounding = False
    with torch.no_grad():  # weights large enough that every layer matters
        for c in m.cross:
            c.weight.mul_(scale_cross)
        for p in m.mlp.parameters():
            p.mul_(scale_mlp)
        m.embeddings.weight.mul_(5.0)
    r = RefDCNv2(nums, 13, 16, 3, (400, 400), dtype=torch.float64)
    with torch.no_grad():
        for f in range(26):
            r.emb[f].weight.copy_(m.embeddings.table(f).double().cpu())
        for a, b_ in zip(list(m.cross) + [x for x in m.mlp.modules() if isinstance(x, nn.Linear)]
                         + [m.prediction],
                         list(r.cross) + [x for x in r.mlp.modules() if isinstance(x, nn.Linear)]
                         + [r.out]):
            b_.weight.copy_(a.weight.double().cpu())
            b_.bias.copy_(a.bias.double().cpu())
    return m, r, sparse, dense, nums


@pytest.mark.parametrize("emb_dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_c3_dcnv2_train_step_matches_oracle_model(gpu, emb_dtype):
    """One DCN-v2 train step at the C3 shape (26 x 38,462 rows, D = 16, 13 dense,
    3 cross layers of 429, deep 400-400, B = 4096, plain SGD fused into every
    backward kernel) against RefDCNv2 (the reference-path torch model, fp64) from
    identical weights: the loss and every parameter's UPDATE.  Tables fp32 (the
    reference's dtype: the update is not hidden by table rounding) and bf16 (what
    the C3 bench line runs: RNE table rounding, lr 1e4 so the table updates are
    tens of bf16 ulps and the emulation's tables are rounded the same way); x0 and
    the towers are bf16.  At this shape bf16 storage alone moves the gradients by several percent
    (the 400-wide ReLU layers sum ~400 terms with heavy cancellation): the same
    model in torch fp32 with bf16 rounding at the build's storage points
    (``RefDCNv2(bf16_points=True)``, run here on the GPU) is 5-8 % (L2) and
    10-20 % (max) away from fp64 on the table updates.  So the bar is relative to
    that: the kernels' error against fp64 may not exceed 1.5x the emulation's
    (+1 % of the update), i.e. the HIP path is as accurate as bf16 storage
    allows; the loss within 2e-3."""
    import torch.nn as nn
    from oracle.models import RefDCNv2, criteo_batch, sgd_train_step
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    bf16 = emb_dtype == torch.bfloat16
    # table updates well above the tables' resolution (bf16: ~40 ulps median)
    B, lr = 4096, (1e4 if bf16 else 1.0)
    m, r, sparse, dense, nums = _dcnv2_pair(gpu, 38462, B, emb_dtype=emb_dtype)
    assert m.embeddings.weight.dtype == emb_dtype
    ids, dn, label = criteo_batch(nums, B, seed=0)
    data = {c.feature_name: ids[:, f].to(torch.int32).to(gpu) for f, c in enumerate(sparse)}
    data.update({c.feature_name: dn[:, j].to(gpu) for j, c in enumerate(dense)})
    data["label"] = label.to(gpu)
    before_state = [v.clone() for v in r.state_dict().values()]
    before_t = [r.emb[f].weight.detach().clone() for f in range(26)]
    rl = list(r.cross) + [x for x in r.mlp.modules() if isinstance(x, nn.Linear)] + [r.out]
    before_l = [(x.weight.detach().clone(), x.bias.detach().clone()) for x in rl]
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), BCEWithLogitsLoss(), [], gpu)
    assert m.embeddings.update == "sgd"
    loss = float(m.train_step(data)["loss"])
    rloss = float(sgd_train_step(r, torch.optim.SGD(r.parameters(), lr=lr), ids, dn.double(),
                                 label))
    assert abs(loss - rloss) <= 2e-3 * max(1.0, abs(rloss)), (loss, rloss)
    # the bf16-storage emulation (fp32 + bf16 rounding points), from the same weights
    e = RefDCNv2(nums, 13, 16, 3, (400, 400), dtype=torch.float32, bf16_points=True)
    e.load_state_dict(dict(zip(e.state_dict(), before_state)))
    e = e.to(gpu)
    sgd_train_step(e, torch.optim.SGD(e.parameters(), lr=lr), ids.to(gpu), dn.to(gpu),
                   label.to(gpu))
    el = list(e.cross) + [x for x in e.mlp.modules() if isinstance(x, nn.Linear)] + [e.out]

    def upd_close(got_after, emu_after, want_after, before, name):
        dg = got_after.double().cpu() - before
        de = emu_after.double().cpu() - before
        dw = want_after.double() - before
        assert float(dw.abs().max()) > 0, name
        for norm in (lambda t: float(t.norm()), lambda t: float(t.abs().max())):
            eg, ee = norm(dg - dw), norm(de - dw)
            assert eg <= 1.5 * ee + 0.01 * norm(dw), (name, eg / norm(dw), ee / norm(dw))

    rnd = (lambda t: t.detach().to(torch.bfloat16)) if bf16 else (lambda t: t.detach())  # noqa: E731
    for f in range(26):
        upd_close(m.embeddings.table(f).detach(), rnd(e.emb[f].weight),
                  r.emb[f].weight.detach(), before_t[f], f"table{f}")
    ml = list(m.cross) + [x for x in m.mlp.modules() if isinstance(x, nn.Linear)] + [m.prediction]
    for i, (a, b_, c_) in enumerate(zip(ml, rl, el)):
        upd_close(a.weight.detach(), c_.weight.detach(), b_.weight.detach(), before_l[i][0], f"W{i}")
        upd_close(a.bias.detach(), c_.bias.detach(), b_.bias.detach(), before_l[i][1], f"b{i}")


# ---------------------------------------------------------------------------
# C5 indexing: element offsets past 2^31
# ---------------------------------------------------------------------------

def test_c5_rows_past_2_31_gather_and_fused_sgd(gpu):
    """A bf16 bank of 3 x 30 M rows with the packed first-order column (64-B rows,
    5.76 GB): the table-2 rows used sit at elements 2.87e9-2.88e9, i.e. element
    offsets > 2^31 and byte offsets > 2^32 (the C5 100M-row tables have them
    from table 1 on).  Forward: the interaction kernel's x0 is a bit copy of
    the looked-up rows.  Backward: fused row-sparse SGD (RNE) on those rows within
    1 bf16 ulp of the oracle's dense SGD; untouched rows keep their bits."""
    from pytorchrec_amd.embedding import EmbeddingBank, interact
    R, D, B, lr = 30_000_000, 16, 4096, 0.5
    bank = EmbeddingBank([R, R, R], D, with_first_order=True, dtype=torch.bfloat16,
                         update="sgd", device=gpu)
    bank.use_fused_sgd(lr)
    bank.stochastic_rounding = False
    assert (bank.row_offset[2] + R - 300_000) * bank.row_stride > 2 ** 31  # every table-2 row used
    assert (bank.total_rows - 1) * bank.row_stride * 2 > 2 ** 32
    rng = np.random.default_rng(55)
    ids_np = np.stack([rng.integers(0, R, B), rng.integers(R - 1000, R, B),
                       rng.integers(R - 300_000, R, B)], 1)
    ids_np[:4, 2] = [R - 1, R - 1, 0, R - 300_000]  # last row twice, first row
    ids_np[4:40, 2] = R - 7  # a hot row
    with torch.no_grad():
        bank.weight.zero_()
        rows = np.unique(np.concatenate([bank.row_offset[f] + ids_np[:, f] for f in range(3)]))
        vals = (rng.standard_normal((rows.size, D + 1)) * 0.5).astype(np.float32)
        vbits = ref.f32_to_bf16_bits(vals)
        ridx = torch.from_numpy(rows).to(gpu)
        bank.weight[ridx, :D + 1] = torch.from_numpy(vbits.view(np.int16)).view(
            torch.bfloat16).to(gpu)
    tables_rows = {int(r): vbits[i] for i, r in enumerate(rows)}
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(3)]
    x0, logit = interact(bank, ids, fm2=True, first_order=True, x0_cols=3 * D,
                         x0_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    x0_bits = x0.detach().cpu().view(torch.int16).numpy().view(np.uint16).reshape(B, 3, D)
    want_bits = np.stack([np.stack([tables_rows[bank.row_offset[f] + int(i)][:D]
                                    for i in ids_np[:, f]]) for f in range(3)], 1)
    assert np.array_equal(x0_bits, want_bits), "gather past 2^31 is not a bit copy"

    dx0 = (rng.standard_normal((B, 3 * D)) * 0.05).astype(np.float32)
    dlogit = (rng.standard_normal(B) * 0.05).astype(np.float32)
    torch.autograd.backward([x0, logit], [torch.from_numpy(dx0).to(gpu).to(torch.bfloat16),
                                          torch.from_numpy(dlogit).to(gpu)])
    torch.cuda.synchronize()
    v = ref.bf16_bits_to_f32(want_bits).astype(np.float64)
    gv = ref.bf16_round(dx0).reshape(B, 3, D) + ref.fm2_bwd(v, dlogit)
    after = bank.weight[ridx, :D + 1].detach().cpu().view(torch.int16).numpy().view(np.uint16)
    pos = {int(r): i for i, r in enumerate(rows)}
    for f in range(3):
        uniq = np.unique(ids_np[:, f])
        tab = np.stack([ref.bf16_bits_to_f32(tables_rows[bank.row_offset[f] + int(u)])
                        for u in uniq]).astype(np.float64)
        remap = np.searchsorted(uniq, ids_np[:, f])
        want_v = ref.sgd_rows(tab[:, :D], remap, gv[:, f], lr)
        want_w = ref.sgd_rows(tab[:, D:], remap, dlogit[:, None], lr)
        got = after[[pos[bank.row_offset[f] + int(u)] for u in uniq]]
        assert _ulp_close(got[:, :D], want_v).all(), f"table {f}: SGD past 2^31 off by > 1 ulp"
        assert _ulp_close(got[:, D:D + 1], want_w).all(), f"table {f}: first-order SGD"
    # a sample of untouched rows (never written) is still zero
    probe = torch.tensor([bank.total_rows - 2, bank.row_offset[2] + R // 2, 12345], device=gpu)
    touched = set(rows.tolist())
    probe = probe[[int(p) not in touched for p in probe.tolist()]]
    assert torch.count_nonzero(bank.weight[probe].float()) == 0
    del bank
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# FunkSVD (the reference's registered model) against the reference's own outputs
# ---------------------------------------------------------------------------

def _funk(gpu=None):
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.model import FunkSVD
    ucol = CategoricalColumnWithIdentity(50, "uid")
    icol = CategoricalColumnWithIdentity(37, "iid")
    lcol = CategoricalColumnWithIdentity(2, "label")
    m = FunkSVD(ucol, icol, lcol, emb_size=8, random_seed=2020)
    return m.to(gpu) if gpu is not None else m


def test_funksvd_train_step_matches_reference_g10(gpu):
    """The product FunkSVD (seed 2020: bit-identical init to the reference's, checked
    against G10's 'before' tables) takes one IModel.train_step on the GPU with MSE
    loss and SGD(lr 0.5) (dense grad in the reference, fused row-sparse SGD here)
    and must land on the reference's own 'after' tables (fp32) within 1e-5."""
    g = golden("g10_funksvd_sgd_step.npz")
    m = _funk()
    sd = m.state_dict()
    assert np.array_equal(sd["u_embeddings.weight"].numpy().view(np.uint32),
                          g["u_before"].view(np.uint32))
    assert np.array_equal(sd["i_embeddings.weight"].numpy().view(np.uint32),
                          g["i_before"].view(np.uint32))
    lr = float(g["lr"])
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), torch.nn.MSELoss(), [], gpu)
    assert m.embeddings.update == "sgd"
    batch = {"uid": torch.from_numpy(g["uid"]), "iid": torch.from_numpy(g["iid"]),
             "label": torch.from_numpy(g["label"])}
    loss = float(m.train_step(batch)["loss"])
    assert abs(loss - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])), (loss, float(g["loss"]))
    sd = m.state_dict()
    for key, want in (("u_embeddings.weight", g["u_after"]), ("i_embeddings.weight", g["i_after"])):
        got = sd[key].cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-8, err_msg=key)
    untouched = np.setdiff1d(np.arange(50), g["uid"])
    assert np.array_equal(sd["u_embeddings.weight"].cpu().numpy()[untouched].view(np.uint32),
                          g["u_after"][untouched].view(np.uint32))


def test_funksvd_sampled_branch_matches_reference_g11(gpu):
    """FunkSVD.py:56-65 on the GPU: prediction [B, N] and the [1, 0, ...] target,
    reference tables loaded under the reference's keys."""
    g = golden("g11_funksvd_sampled.npz")
    m = _funk()
    m.load_state_dict({"u_embeddings.weight": torch.from_numpy(g["u_table"]),
                       "i_embeddings.weight": torch.from_numpy(g["i_table"])})
    m = m.to(gpu).eval()
    with torch.no_grad():
        pred, tgt = m({"uid": torch.from_numpy(g["uid"]).to(gpu),
                       "iid": torch.from_numpy(g["iid"]).to(gpu)})
    assert pred.shape == g["prediction"].shape and tgt.dtype == torch.float32
    u = g["u_table"].astype(np.float64)[g["uid"]]
    i = g["i_table"].astype(np.float64)[g["iid"]]
    mag = (np.abs(u[:, None, :]) * np.abs(i)).sum(-1)
    assert np.all(np.abs(pred.cpu().numpy() - g["prediction"]) <= 1e-5 * (mag + 1e-30))
    assert np.array_equal(tgt.cpu().numpy(), g["target"])


def test_funksvd_sampled_branch_trains(gpu):
    """The sampled branch's backward: every (sample, candidate) pair scatters into
    its user and item rows (repeated users / candidates summed)."""
    g = golden("g11_funksvd_sampled.npz")
    m = _funk()
    m.load_state_dict({"u_embeddings.weight": torch.from_numpy(g["u_table"]),
                       "i_embeddings.weight": torch.from_numpy(g["i_table"])})
    lr = 0.5
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), torch.nn.MSELoss(), [], gpu)
    m.train_step({"uid": torch.from_numpy(g["uid"]), "iid": torch.from_numpy(g["iid"])})
    u0 = g["u_table"].astype(np.float64)
    i0 = g["i_table"].astype(np.float64)
    uid, iid = g["uid"], g["iid"]
    B, N = iid.shape
    pred = (u0[uid][:, None, :] * i0[iid]).sum(-1)
    dpred = 2.0 * (pred - g["target"]) / pred.size
    uu = np.repeat(uid, N)
    want_u = ref.sgd_rows(u0, uu, (dpred[..., None] * i0[iid]).reshape(B * N, -1), lr)
    want_i = ref.sgd_rows(i0, iid.reshape(-1), (dpred[..., None] * u0[uid][:, None, :]).reshape(
        B * N, -1), lr)
    sd = m.state_dict()
    np.testing.assert_allclose(sd["u_embeddings.weight"].cpu().numpy(), want_u, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(sd["i_embeddings.weight"].cpu().numpy(), want_i, rtol=1e-5, atol=1e-8)


# ---------------------------------------------------------------------------
# DIN pooling kernels in isolation (fp32 arithmetic)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("L,E", [(50, 16), (50, 32), (7, 8), (64, 16)])
def test_din_pool_kernels_isolated_fp32(gpu, L, E):
    """mrec_din_pool_fwd / _bwd given the scores: attention weights a (fp32) within
    1e-5 of ref.din_softmax_pool; the pooled u (rounded once to bf16 in the top
    input) within 1 bf16 ulp of the fp64 value; ds and dk (fp32) within 1e-5 of
    ref.din_softmax_pool_bwd relative to their magnitudes.  Padded positions
    (history id 0, position 0 always valid, utils.py:5-10) get a = 0."""
    from pytorchrec_amd import _mrec, dense as Dn
    B = 300
    rng = np.random.default_rng(L * 100 + E)
    s = (rng.standard_normal(B * L) * 3).astype(np.float32)
    lens = rng.integers(1, L + 1, B)
    lens[:3] = [1, L, 1]
    his = rng.integers(1, 1000, (B, L)).astype(np.int32)
    his[np.arange(L)[None, :] >= lens[:, None]] = 0
    his[2, 0] = 0  # position 0 stays valid even when its id is PAD
    q = ref.f32_to_bf16_bits(rng.standard_normal((B, E)).astype(np.float32))
    k = ref.f32_to_bf16_bits(rng.standard_normal((B * L, E)).astype(np.float32))
    t = lambda a: torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).to(gpu)  # noqa: E731
    qg, kg = Dn._bf16_rows(t(q)), Dn._bf16_rows(t(k))
    sg = torch.from_numpy(s).to(gpu)
    hg = torch.from_numpy(his).to(gpu)
    a = torch.empty(B, L, dtype=torch.float32, device=gpu)
    top = Dn._alloc(B, 2 * E, torch.bfloat16, gpu)
    _mrec.call("mrec_din_pool_fwd", sg.data_ptr(), 1, hg.data_ptr(), hg.stride(0), qg.data_ptr(),
               qg.stride(0), kg.data_ptr(), kg.stride(0), B, L, E, a.data_ptr(), top.data_ptr(),
               top.stride(0), _mrec.stream_handle())
    valid = ref.valid_his_index(his)
    kf = ref.bf16_bits_to_f32(k).astype(np.float64).reshape(B, L, E)
    u, a_ref = ref.din_softmax_pool(s.reshape(B, L), valid, kf)
    a_got = a.cpu().numpy()
    assert np.all(np.abs(a_got - a_ref) <= 1e-5 * a_ref + 1e-12)
    assert np.all(a_got[valid == 0] == 0)
    top_bits = top.detach().cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(top_bits[:, :E], q)
    umag = (a_ref[..., None] * np.abs(kf)).sum(1)
    got_u = ref.bf16_bits_to_f32(top_bits[:, E:2 * E]).astype(np.float64)
    assert np.all(np.abs(got_u - u) <= ref.bf16_ulp(u) * 0.5001 + 1e-5 * umag)

    du = ref.f32_to_bf16_bits((rng.standard_normal((B, E))).astype(np.float32))
    dtop = np.zeros((B, 2 * E), np.uint16)
    dtop[:, E:] = du
    dtg = Dn._bf16_rows(t(dtop))
    ds = torch.empty(B * L, dtype=torch.float32, device=gpu)
    dk = torch.empty(B * L, E, dtype=torch.float32, device=gpu)
    _mrec.call("mrec_din_pool_bwd", dtg.data_ptr(), dtg.stride(0), a.data_ptr(), kg.data_ptr(),
               kg.stride(0), B, L, E, ds.data_ptr(), dk.data_ptr(), dk.stride(0),
               _mrec.stream_handle())
    duf = ref.bf16_bits_to_f32(du).astype(np.float64)
    ds_ref, dk_ref = ref.din_softmax_pool_bwd(a_got, kf, duf)
    gmag = (np.abs(kf) * np.abs(duf)[:, None, :]).sum(-1)
    ds_mag = a_got * (gmag + (a_got * gmag).sum(-1, keepdims=True))
    assert np.all(np.abs(ds.cpu().numpy().reshape(B, L) - ds_ref) <= 1e-5 * ds_mag + 1e-12)
    dk_got = dk.cpu().numpy().reshape(B, L, E)
    assert np.all(np.abs(dk_got - dk_ref) <= 1e-6 * np.abs(dk_ref) + 1e-12)


# ---------------------------------------------------------------------------
# FM (config C1's model) on the GPU: every operand fp32 -> a tight full-step pin
# ---------------------------------------------------------------------------

def test_fm_train_step_on_gpu_matches_oracle_model_fp32_tight(gpu):
    """One FM train step (C1 model: MovieLens-1M-shaped 24 fields, D = 16, fp32
    tables, B = 4096, BCE, SGD fused into the embedding backward) on the GPU
    against the reference-path model (RefDeepFM(deep=False): 24 nn.Embedding +
    24 Embedding(rows, 1) + global bias, fp64).  No bf16 anywhere: loss within
    1e-6, every updated table value within 2 fp32 ulps of the fp64 result plus
    1e-5 of the update (first-order weights likewise)."""
    from oracle.models import RefDeepFM, sgd_train_step
    from pytorchrec_amd.console_main import ML1M_FIELDS, synthetic_ml1m
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.model import FM
    cols = [CategoricalColumnWithIdentity(card, f"c_c_{name}") for name, card in ML1M_FIELDS]
    lab = CategoricalColumnWithIdentity(2, "label")
    m = FM(cols, lab, emb_size=16, emb_dtype=torch.float32, device=gpu, random_seed=5)
    with torch.no_grad():
        m.embeddings.weight.mul_(10.0)  # FM term of the same order as the first order
    nums = [c for _, c in ML1M_FIELDS]
    r = RefDeepFM(nums, 0, 16, deep=False, dtype=torch.float64)
    with torch.no_grad():
        for f in range(len(nums)):
            r.emb[f].weight.copy_(m.embeddings.table(f).double().cpu())
            r.w1[f].weight.copy_(m.embeddings.first_order(f).double().cpu()[:, None])
        r.global_bias.copy_(m.global_bias.double().cpu())
    data = synthetic_ml1m(4096, seed=3)
    ids = torch.stack([data[c.feature_name].long() for c in cols], 1)
    label = data["label"].double()
    lr = 20.0
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), BCEWithLogitsLoss(), [], gpu)
    assert m.embeddings.update == "sgd"
    before = [(r.emb[f].weight.detach().clone(), r.w1[f].weight.detach()[:, 0].clone())
              for f in range(len(nums))]
    loss = float(m.train_step({k: v.to(gpu) for k, v in data.items()})["loss"].detach())
    rloss = float(sgd_train_step(r, torch.optim.SGD(r.parameters(), lr=lr), ids, None, label))
    assert abs(loss - rloss) <= 1e-6 * abs(rloss), (loss, rloss)
    ulp = lambda x: np.spacing(np.abs(x).astype(np.float32)).astype(np.float64)  # noqa: E731
    for f in range(len(nums)):
        for got, want, b0 in ((m.embeddings.table(f), r.emb[f].weight, before[f][0]),
                              (m.embeddings.first_order(f), r.w1[f].weight[:, 0], before[f][1])):
            got = got.detach().double().cpu().numpy()
            want = want.detach().numpy()
            upd = np.abs(want - b0.numpy()).max()
            assert upd > 0, f
            err = np.abs(got - want)
            assert np.all(err <= 2 * ulp(want) + 1e-5 * upd), (f, float((err / upd).max()))
    assert abs(float(m.global_bias) - float(r.global_bias)) <= 1e-6 * max(1e-3, abs(float(r.global_bias)))


# ---------------------------------------------------------------------------
# C2: the DeepFM train step at the config shape
# ---------------------------------------------------------------------------

def test_c2_deepfm_train_step_matches_oracle_model(gpu):
    """One DeepFM train step at the C2 shape (26 x 38,462 rows, D = 16 bf16 tables
    with the packed first-order column, 13 dense, MLP 400-400-400, B = 4096, plain
    SGD fused into every backward kernel, RNE table rounding) against RefDeepFM
    (the reference-path torch model, fp64) from identical weights: the loss and
    every parameter's UPDATE.  The bar is relative to what bf16 storage alone costs
    (as in the C3 test): ``RefDeepFM(bf16_points=True)`` in fp32 on the GPU, its
    tables rounded to bf16 after the step like the bank's, is 2-4 % (L2) away from
    fp64 on the table updates; the kernels' error against fp64 may not exceed 1.5x
    the emulation's + 1 % of the update.  Weights are scaled up so every term of
    the logit moves the gradients, and lr = 100 makes the table updates ~10-100
    bf16 ulps."""
    import torch.nn as nn
    from oracle.models import RefDeepFM, criteo_batch, sgd_train_step
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.model import DeepFM
    B, lr, rows = 4096, 100.0, 38462
    nums = [rows] * 26
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{f + 1}") for f, n in enumerate(nums)]
    dense = [NumericColumn(f"c_n_I{j + 1}") for j in range(13)]
    lab = CategoricalColumnWithIdentity(2, "label")
    m = DeepFM(sparse, dense, lab, emb_size=16, layers=(400, 400, 400), dropout=0.0,
               emb_dtype=torch.bfloat16, device=gpu, random_seed=2020)
    r = RefDeepFM(nums, 13, 16, (400, 400, 400), dtype=torch.float64)
    with torch.no_grad():
        for p in list(r.mlp.parameters()) + [r.out.weight]:
            p.mul_(6.0)
        for f in range(26):  # bf16-representable tables, shared by all three models
            r.emb[f].weight.copy_((r.emb[f].weight * 5.0).to(torch.bfloat16).double())
            r.w1[f].weight.copy_((r.w1[f].weight * 5.0).to(torch.bfloat16).double())
            m.embeddings.table(f).copy_(r.emb[f].weight.to(gpu))
            m.embeddings.first_order(f).copy_(r.w1[f].weight[:, 0].to(gpu))
        m.dense_weight.copy_(r.dense_w.weight[0].to(gpu))
        m.global_bias.copy_(r.global_bias.to(gpu))
        ml = [x for x in m.mlp.modules() if isinstance(x, nn.Linear)] + [m.prediction]
        rl = [x for x in r.mlp.modules() if isinstance(x, nn.Linear)] + [r.out]
        for a, b_ in zip(ml, rl):
            a.weight.copy_(b_.weight.to(gpu))
            a.bias.copy_(b_.bias.to(gpu))
    m.embeddings.stochastic_rounding = False
    before_state = [v.clone() for v in r.state_dict().values()]
    before_t = [(r.emb[f].weight.detach().clone(), r.w1[f].weight.detach()[:, 0].clone())
                for f in range(26)]
    before_l = [(x.weight.detach().clone(), x.bias.detach().clone()) for x in rl]
    before_lin = (r.dense_w.weight.detach()[0].clone(), r.global_bias.detach().clone())
    ids, dn, label = criteo_batch(nums, B, seed=0)
    data = {c.feature_name: ids[:, f].to(torch.int32).to(gpu) for f, c in enumerate(sparse)}
    data.update({c.feature_name: dn[:, j].to(gpu) for j, c in enumerate(dense)})
    data["label"] = label.to(gpu)
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), BCEWithLogitsLoss(), [], gpu)
    assert m.embeddings.update == "sgd"
    assert m.embeddings.weight.dtype == torch.bfloat16
    loss = float(m.train_step(data)["loss"].detach())
    rloss = float(sgd_train_step(r, torch.optim.SGD(r.parameters(), lr=lr), ids, dn.double(),
                                 label).detach())
    assert abs(loss - rloss) <= 2e-3 * max(1.0, abs(rloss)), (loss, rloss)
    e = RefDeepFM(nums, 13, 16, (400, 400, 400), dtype=torch.float32, bf16_points=True)
    e.load_state_dict(dict(zip(e.state_dict(), before_state)))
    e = e.to(gpu)
    sgd_train_step(e, torch.optim.SGD(e.parameters(), lr=lr), ids.to(gpu), dn.to(gpu),
                   label.to(gpu))

    def upd_close(got_after, emu_after, want_after, before, name):
        dg = got_after.double().cpu() - before
        de = emu_after.double().cpu() - before
        dw = want_after.double() - before
        assert float(dw.abs().max()) > 0, name
        for norm in (lambda t: float(t.norm()), lambda t: float(t.abs().max())):
            eg, ee = norm(dg - dw), norm(de - dw)
            assert eg <= 1.5 * ee + 0.01 * norm(dw), (name, eg / norm(dw), ee / norm(dw))

    rnd = lambda t: t.detach().to(torch.bfloat16)  # noqa: E731  the bank's rounding
    for f in range(26):
        upd_close(m.embeddings.table(f).detach(), rnd(e.emb[f].weight),
                  r.emb[f].weight.detach(), before_t[f][0], f"table{f}")
        upd_close(m.embeddings.first_order(f).detach(), rnd(e.w1[f].weight[:, 0]),
                  r.w1[f].weight.detach()[:, 0], before_t[f][1], f"w{f}")
    el = [x for x in e.mlp.modules() if isinstance(x, nn.Linear)] + [e.out]
    for i, (a, b_, c_) in enumerate(zip(ml, rl, el)):
        upd_close(a.weight.detach(), c_.weight.detach(), b_.weight.detach(), before_l[i][0], f"W{i}")
        upd_close(a.bias.detach(), c_.bias.detach(), b_.bias.detach(), before_l[i][1], f"b{i}")
    upd_close(m.dense_weight.detach(), e.dense_w.weight.detach()[0], r.dense_w.weight.detach()[0],
              before_lin[0], "dense_w")
    upd_close(m.global_bias.detach(), e.global_bias.detach(), r.global_bias.detach(),
              before_lin[1], "global_bias")


# ---------------------------------------------------------------------------
# A2 / A3 product columns on cuda tensors against the reference's G8
# ---------------------------------------------------------------------------

def test_columns_on_cuda_match_reference_g8(gpu):
    """CrossedColumn (CrossedColumn.py:14-27) and NumericColumn (NumericColumn.py:25-34)
    fed cuda tensors: the crossed ids bit-exact vs G8 (int64, on the device), then
    gathered from a bank of category_num rows by the HIP gather (bit copy of the
    looked-up rows); the three normalisations bit-exact vs G8 (fp32 IEEE
    subtract / divide on the device, same operation order as the reference)."""
    from pytorchrec_amd.embedding import EmbeddingBank, gather
    from pytorchrec_amd.feature_column import (CategoricalColumnWithIdentity, CrossedColumn,
                                               NormalizationMode, NumericColumn)
    g = golden("g8_columns.npz")
    cols = [CategoricalColumnWithIdentity(7, "a"), CategoricalColumnWithIdentity(5, "b"),
            CategoricalColumnWithIdentity(3, "c")]
    cross = CrossedColumn(cols)
    batch = {k: torch.from_numpy(g[k]).to(gpu) for k in ("a", "b", "c")}
    ids = cross.get_feature_ids(batch)
    assert ids.is_cuda and ids.dtype == torch.int64
    assert np.array_equal(ids.cpu().numpy(), g["crossed"])
    bank = EmbeddingBank([cross.category_num], 16, dtype=torch.float32, device=gpu)
    with torch.no_grad():
        bank.weight.normal_(0, 1)
    out = gather(bank, [ids])
    torch.cuda.synchronize()
    want = bank.table(0).detach().cpu().numpy()[g["crossed"]]
    assert np.array_equal(out.detach().cpu().numpy().reshape(want.shape).view(np.uint32),
                          want.view(np.uint32))
    num = NumericColumn("x", min_value=-3.0, max_value=7.0, mean_value=2.0, std_value=2.9)
    xb = {"x": torch.from_numpy(g["x"]).to(gpu)}
    for mode, key in ((NormalizationMode.NOP, "nop"), (NormalizationMode.MAX_MIN, "max_min"),
                      (NormalizationMode.Z_SCORE, "z_score")):
        got = num.get_feature_data(xb, mode)
        assert got.is_cuda and got.dtype == torch.float32
        assert np.array_equal(got.cpu().numpy().view(np.uint32), g[key].view(np.uint32)), key


# ---------------------------------------------------------------------------
# C4: the composed DIN train step at the config shape
# ---------------------------------------------------------------------------

def test_c4_din_train_step_matches_oracle_model(gpu, monkeypatch):
    """One DIN train step at the C4 shape (item 63,001 + PAD / category 801 + PAD
    bf16 tables, D = 16, L = 50 with lengths U{1..50}, attention MLP 80-40-1, top
    MLP 200-80-1, B = 4096, plain SGD, RNE table rounding) on the PRODUCT path --
    ``mrec_din_gather`` (lookup ids with padding slots built in the gather launch),
    the fused attention unit (``mrec_din_att_fwd`` / ``_bwd`` / ``_wgrad`` with the
    fused SGD of the attention MLP), the fused top tower with its deferred dW
    reductions riding in the bucketed embedding-backward launch
    (``mrec_emb_bwd_large_fused_ex`` with jobs), and the bucketed fused SGD of the
    tables -- against RefDIN (the reference-path torch model, fp64) from identical
    weights: the loss and every parameter's UPDATE.

    The bar is the C2 / C3 one: ``RefDIN(bf16_points=True)`` in fp32 on the GPU
    (bf16 at the build's storage points, its tables rounded to bf16 after the step
    like the bank's) sets what bf16 storage alone costs (tables 3-6 % L2, the
    attention MLP 1-3 %, the top tower 0.1-1 %); the kernels' error against fp64
    may not exceed 1.5x the emulation's + 1 % of the update.  Scales: attention
    weights x40 and rows x10 (scores spread ~1.6 std: a peaked, not uniform,
    softmax, so every term of the unit's backward matters), top tower x6, lr 1e5
    (table updates ~20 bf16 ulps median).  The attention output bias gets an
    analytically zero gradient (sum_j ds_j = 0): its update is bounded by 1e-4 of
    the score weights' update."""
    import torch.nn as nn
    from oracle.models import RefDIN, din_batch, sgd_train_step
    from pytorchrec_amd import _mrec
    from pytorchrec_amd import dense as D
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.model import DIN
    B, L, lr, ITEMS, CATES = 4096, 50, 1e5, 63002, 802
    cols = [CategoricalColumnWithIdentity(ITEMS, "iid"), CategoricalColumnWithIdentity(CATES, "cid"),
            CategoricalColumnWithIdentity(ITEMS, "pos_his"),
            CategoricalColumnWithIdentity(CATES, "pos_his_cate")]
    m = DIN(*cols, CategoricalColumnWithIdentity(2, "label"), emb_size=16, att_layers=(80, 40),
            layers=(200, 80), emb_dtype=torch.bfloat16, device=gpu, random_seed=2020)
    m.embeddings.stochastic_rounding = False
    r = RefDIN(ITEMS, CATES, 16, (80, 40), (200, 80), dtype=torch.float64)
    with torch.no_grad():
        for p in list(r.att_mlp.parameters()) + list(r.att_out.parameters()):
            p.mul_(40.0)
        for p in list(r.mlp.parameters()) + [r.out.weight]:
            p.mul_(6.0)
        for t in (r.item, r.cate):  # bf16-representable tables shared by all three models
            t.weight.copy_((t.weight * 10.0).to(torch.bfloat16).double())
        m.embeddings.table(0).copy_(r.item.weight.to(gpu))
        m.embeddings.table(1).copy_(r.cate.weight.to(gpu))
    pairs = [(a, b_) for a, b_ in zip(
        [x for x in m.att_mlp.modules() if isinstance(x, nn.Linear)] + [m.att_out]
        + [x for x in m.mlp.modules() if isinstance(x, nn.Linear)] + [m.prediction],
        [x for x in r.att_mlp.modules() if isinstance(x, nn.Linear)] + [r.att_out]
        + [x for x in r.mlp.modules() if isinstance(x, nn.Linear)] + [r.out])]
    assert len(pairs) == 6
    with torch.no_grad():
        for a, b_ in pairs:
            a.weight.copy_(b_.weight.to(gpu))
            a.bias.copy_(b_.bias.to(gpu))
    before_state = [v.clone() for v in r.state_dict().values()]
    before_t = [r.item.weight.detach().clone(), r.cate.weight.detach().clone()]
    before_l = [(b_.weight.detach().clone(), b_.bias.detach().clone()) for _, b_ in pairs]
    iid, cid, his, hcat, label = din_batch(ITEMS, CATES, B, L, seed=0)
    data = {"iid": iid.to(torch.int32).to(gpu), "cid": cid.to(torch.int32).to(gpu),
            "pos_his": his.to(torch.int32).to(gpu), "pos_his_cate": hcat.to(torch.int32).to(gpu),
            "label": label.to(gpu)}
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), BCEWithLogitsLoss(), [], gpu)
    assert m.embeddings.update == "sgd" and m.embeddings.weight.dtype == torch.bfloat16
    assert D.DIN_FUSED and D.din_att_supported(32, m.att_mlp, m.att_out)
    calls = []
    real_call = _mrec.call

    def spy(name, *args):
        calls.append((name, args))
        return real_call(name, *args)

    monkeypatch.setattr(_mrec, "call", spy)
    loss = float(m.train_step(data)["loss"].detach())
    torch.cuda.synchronize()
    monkeypatch.setattr(_mrec, "call", real_call)
    names = [n for n, _ in calls]
    for want in ("mrec_din_gather", "mrec_din_att_fwd", "mrec_din_att_bwd", "mrec_din_att_wgrad",
                 "mrec_emb_bwd_large_fused_ex"):
        assert want in names, (want, names)
    ex = [a for n, a in calls if n == "mrec_emb_bwd_large_fused_ex"]
    assert len(ex) == 1 and ex[0][-3] > 0, "the top tower's dW reductions must ride in the bucket launch"
    # the attention MLP took its fused SGD in place (no gradient handed back)
    wg = [a for n, a in calls if n == "mrec_din_att_wgrad"]
    assert wg[0][5] is None and wg[0][6] == lr
    rloss = float(sgd_train_step(r, torch.optim.SGD(r.parameters(), lr=lr),
                                 (iid, cid, his, hcat), None, label.double()).detach())
    assert abs(loss - rloss) <= 2e-3 * max(1.0, abs(rloss)), (loss, rloss)
    e = RefDIN(ITEMS, CATES, 16, (80, 40), (200, 80), dtype=torch.float32, bf16_points=True)
    e.load_state_dict(dict(zip(e.state_dict(), before_state)))
    e = e.to(gpu)
    sgd_train_step(e, torch.optim.SGD(e.parameters(), lr=lr),
                   tuple(t.to(gpu) for t in (iid, cid, his, hcat)), None, label.to(gpu))

    def upd_close(got_after, emu_after, want_after, before, name):
        dg = got_after.double().cpu() - before
        de = emu_after.double().cpu() - before
        dw = want_after.double() - before
        assert torch.isfinite(dg).all(), name
        assert float(dw.abs().max()) > 0, name
        for norm in (lambda t: float(t.norm()), lambda t: float(t.abs().max())):
            eg, ee = norm(dg - dw), norm(de - dw)
            assert eg <= 1.5 * ee + 0.01 * norm(dw), (name, eg / norm(dw), ee / norm(dw))

    rnd = lambda t: t.detach().to(torch.bfloat16)  # noqa: E731  the bank's rounding
    upd_close(m.embeddings.table(0).detach(), rnd(e.item.weight), r.item.weight.detach(),
              before_t[0], "item")
    upd_close(m.embeddings.table(1).detach(), rnd(e.cate.weight), r.cate.weight.detach(),
              before_t[1], "cate")
    # PAD rows (id 0) only ever sit at masked positions here (lengths >= 1): no update
    assert torch.equal(m.embeddings.table(0)[0].double().cpu(), before_t[0][0])
    el = ([x for x in e.att_mlp.modules() if isinstance(x, nn.Linear)] + [e.att_out]
          + [x for x in e.mlp.modules() if isinstance(x, nn.Linear)] + [e.out])
    for i, ((a, b_), c_) in enumerate(zip(pairs, el)):
        upd_close(a.weight.detach(), c_.weight.detach(), b_.weight.detach(), before_l[i][0], f"W{i}")
        if i == 2:  # score bias: sum_j ds_j = 0
            db = float((a.bias.detach().double().cpu() - before_l[i][1]).abs().max())
            dw3 = float((b_.weight.detach() - before_l[i][0]).abs().max())
            assert db <= 1e-4 * dw3, (db, dw3)
            continue
        upd_close(a.bias.detach(), c_.bias.detach(), b_.bias.detach(), before_l[i][1], f"b{i}")
