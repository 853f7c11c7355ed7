"""GPU numerics of the MFMA GEMM (libmrec mrec_gemm) and the dense-tower layers
built on it, against plain torch fp64/fp32 references of the same op on the same
bf16-rounded operands.

Tolerance: operands are bf16, accumulation fp32 (error ~1e-6 * sum|a*b|), the
output is rounded once to bf16 (<= 1 ulp = 2^-8 relative) — so the check is
|got - ref| <= 2^-8 * |ref| + 1e-5 * sum_k |a_k b_k| (+1e-30).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float64)


def _close(got, want, mag, out_bf16=True):
    got = got.double().cpu()
    want = want.double().cpu()
    mag = mag.double().cpu()
    tol = (2.0 ** -8 if out_bf16 else 1e-6) * want.abs() + 1e-5 * mag + 1e-30
    bad = (got - want).abs() > tol
    return (~bad).all().item(), ((got - want).abs() / tol).max().item()


@pytest.mark.parametrize("shape", [(300, 77, 93), (4096, 400, 429), (64, 1, 400), (1, 5, 7),
                                   (200, 96, 1000)])
def test_gemm_forward_bias_relu(gpu, shape):
    from pytorchrec_amd import dense as D, _mrec
    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.1).to(gpu)
    b = (torch.randn(N, generator=g) * 0.1).to(gpu)
    xp = torch.zeros(M, D._r8(K), dtype=torch.bfloat16, device=gpu)[:, :K]
    xp.copy_(x)
    wr, _ = D.weight_prep(W, tr=False)
    y = D.gemm(xp, _mrec.LAYOUT_ROW, wr[:, :K], _mrec.LAYOUT_ROW, M, N, K, bias=b,
               act=_mrec.ACT_RELU)
    want = torch.relu(_bf(x) @ _bf(W).T + b.double())
    mag = _bf(x).abs() @ _bf(W).abs().T + b.double().abs()
    ok, worst = _close(y, want, mag)
    assert ok, worst


@pytest.mark.parametrize("split_k", [1, 4, 13])
def test_gemm_weight_grad_col_col_ones_column(gpu, split_k):
    """dW = dZ^T x and db = sum_m dZ via the ones column."""
    from pytorchrec_amd import dense as D, _mrec
    M, N, K = 1000, 70, 45
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(M, N, generator=g).to(torch.bfloat16).to(gpu)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(gpu)
    dy, x = D._bf16_rows(dy), D._bf16_rows(x)  # 16-B aligned rows
    db = torch.empty(N, dtype=torch.float32, device=gpu)
    out = D.gemm(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M, ones_out=db,
                 out_dtype=torch.float32, split_k=split_k)
    dz = _bf(dy)
    want_w = dz.T @ _bf(x)
    want_b = dz.sum(0)
    ok, worst = _close(out[:, :K], want_w, dz.abs().T @ _bf(x).abs(), out_bf16=False)
    assert ok, worst
    ok, worst = _close(db, want_b, dz.abs().sum(0), out_bf16=False)
    assert ok, worst


def _kfrag_np(x):
    """numpy restatement of the k-fragment image (tower_common.h kfrag_idx)."""
    rows, cols = x.shape
    ns, nt = (rows + 31) // 32, (cols + 15) // 16
    img = np.zeros(nt * ns * 512, dtype=x.dtype)
    b, c = np.meshgrid(np.arange(rows), np.arange(cols), indexing="ij")
    idx = (((c >> 4) * ns + (b >> 5)) * 64 + (c & 15) + 16 * ((b & 31) >> 3)) * 8 + (b & 7)
    img[idx.reshape(-1)] = x.reshape(-1)
    return img


@pytest.mark.parametrize("case", ["tower", "ragged"])
def test_tower_dw_kfrag_partials_reduce_to_weight_grads(gpu, case):
    """mrec_tower_dw on k-fragment images (mrec_kfrag_pack, checked bitwise against
    the numpy layout) writes split-K slabs that the generic REDUCE job sums into
    dW = dY^T X and db = sum_b dY, as mrec_gemm would."""
    import ctypes
    from pytorchrec_amd import dense as D, _mrec
    lib = _mrec.lib()
    if case == "tower":
        B, shapes, splits = 4096, [(400, 429), (400, 400), (400, 400)], 5
    else:
        B, shapes, splits = 333, [(77, 50), (200, 129)], 2
    g = torch.Generator().manual_seed(23)
    a = _mrec.TowerDwArgs()
    a.n_layers, a.batch, a.splits = len(shapes), B, splits
    keep, checks = [], []
    for l, (no, ni) in enumerate(shapes):
        dy = D._bf16_rows(torch.randn(B, no, generator=g).to(torch.bfloat16).to(gpu))
        x = D._bf16_rows(torch.randn(B, ni, generator=g).to(torch.bfloat16).to(gpu))
        imgs = []
        for t, n in ((dy, no), (x, ni)):
            im = torch.empty(int(lib.mrec_kfrag_elems(B, n)), dtype=torch.bfloat16, device=gpu)
            _mrec.call("mrec_kfrag_pack", t.data_ptr(), B, n, t.stride(0), im.data_ptr(),
                       _mrec.stream_handle())
            imgs.append(im)
        if l == 0:
            want = _kfrag_np(dy[:, :no].cpu().view(torch.int16).numpy())
            assert np.array_equal(imgs[0].cpu().view(torch.int16).numpy(), want)
        db = torch.empty(no, dtype=torch.float32, device=gpu)
        call = D._Call(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, no, ni, B, _mrec.GEMM_REDUCE,
                       ones_out=db, out_dtype=torch.float32, split_k=splits)
        a.n_out[l], a.n_in[l] = no, ni
        a.dy_img[l], a.x_img[l] = imgs[0].data_ptr(), imgs[1].data_ptr()
        a.ws[l], a.ldws[l] = call.ws.data_ptr(), (ni + 1 + 7) // 8 * 8
        keep += [dy, x, imgs, call]
        dz = _bf(dy)
        checks.append((call, db, dz.T @ _bf(x), dz.sum(0), dz.abs().T @ _bf(x).abs(), dz.abs().sum(0)))
    _mrec.call("mrec_tower_dw", ctypes.byref(a), None, _mrec.stream_handle())
    D._run([c[0] for c in checks])
    torch.cuda.synchronize()
    for c, db, ww, wb, mw, mb in checks:
        ni = ww.shape[1]
        ok, worst = _close(c.out[:, :ni], ww, mw, out_bf16=False)
        assert ok, worst
        ok, worst = _close(db, wb, mb, out_bf16=False)
        assert ok, worst


@pytest.mark.parametrize("masked", [False, True])
def test_gemm_input_grad_row_col_with_zero_pad(gpu, masked):
    """dx = dZ W with W fp32 [N, K] read as a COL operand (== W^T read as ROW);
    columns >= K of the padded output are exactly zero; with an epilogue mask the
    output is zero wherever the mask (a ReLU output) is <= 0."""
    from pytorchrec_amd import dense as D, _mrec
    M, N, K, KX = 513, 400, 429, 432
    g = torch.Generator().manual_seed(9)
    dy = D._bf16_rows(torch.randn(M, N, generator=g).to(torch.bfloat16).to(gpu))
    W = (torch.randn(N, K, generator=g) * 0.05).to(gpu)
    mask = D._alloc(M, KX, torch.bfloat16, gpu)
    mask.copy_(torch.relu(torch.randn(M, KX, generator=g)).to(torch.bfloat16))
    mask[:, :3] = -0.0  # negative zero is not > 0
    wr, wt = D.weight_prep(W)
    mk = mask if masked else None
    # B(k'=n, col=k) = W[n, k]: the row image read as COL, or W^T read as ROW
    dx = D.gemm(dy, _mrec.LAYOUT_ROW, wr, _mrec.LAYOUT_COL, M, KX, N, b_cols=K, mask=mk)
    dx2 = D.gemm(dy, _mrec.LAYOUT_ROW, wt, _mrec.LAYOUT_ROW, M, KX, N, b_cols=K, mask=mk)
    assert torch.equal(dx, dx2)
    want = _bf(dy) @ _bf(W)
    mag = _bf(dy).abs() @ _bf(W).abs()
    if masked:
        keep = mask[:, :K].double() > 0
        assert torch.all(dx[:, :K][~keep] == 0)
        want = want * keep
    ok, worst = _close(dx[:, :K], want, mag)
    assert ok, worst
    assert torch.all(dx[:, K:] == 0)


def test_relu_output_consumed_twice_matches_torch(gpu):
    """A ReLU output feeding two consumers: the gradients accumulate in autograd,
    which voids the consumer's pre-mask stamp, so the producer masks itself."""
    from pytorchrec_amd import dense as D
    g = torch.Generator().manual_seed(3)
    M, K, H = 384, 96, 64
    x = torch.randn(M, K, generator=g)
    W1, b1 = torch.randn(H, K, generator=g) * 0.1, torch.randn(H, generator=g) * 0.1
    W2, W3 = torch.randn(8, H, generator=g) * 0.1, torch.randn(1, H, generator=g) * 0.1
    ps = [t.to(gpu).requires_grad_() for t in (W1, b1, W2, W3)]
    y = D.linear(x.to(gpu).to(torch.bfloat16), ps[0], ps[1], act="relu")
    out = D.linear(y, ps[2], None).float().sum(1) + D.head(y, ps[3], None)
    out.sum().backward()
    rs = [t.double().requires_grad_() for t in (W1, b1, W2, W3)]
    # forward on the bf16-rounded weight (what the GEMM multiplies) so no ReLU flips
    w1 = rs[0] + (_bf(W1) - W1.double())
    yr = torch.relu(_bf(x) @ w1.T + rs[1])
    ((yr @ rs[2].T).sum(1) + (yr @ rs[3].T).reshape(-1)).sum().backward()
    for got, want in zip(ps, rs):
        np.testing.assert_allclose(got.grad.double().cpu().numpy(), want.grad.numpy(),
                                   rtol=3e-2, atol=3e-2 * want.grad.abs().max().item())


def test_head_backward_mask(gpu):
    from pytorchrec_amd import _mrec, dense as D
    g = torch.Generator().manual_seed(4)
    B, H = 1000, 45
    h = D._alloc(B, H, torch.bfloat16, gpu)
    h.copy_(torch.randn(B, H, generator=g).to(torch.bfloat16))
    dz = torch.randn(B, generator=g).to(gpu)
    w = torch.randn(H, generator=g).to(gpu)
    dh = D._alloc(B, H, torch.bfloat16, gpu)
    _mrec.call("mrec_head_bwd", dz.data_ptr(), w.data_ptr(), B, H, h.data_ptr(), h.stride(0),
               dh.data_ptr(), dh.stride(0), _mrec.stream_handle())
    want = (dz[:, None] * w[None, :]) * (h.float() > 0)
    assert torch.equal(dh, want.to(torch.bfloat16))
    assert torch.all(dh.as_strided((B, dh.stride(0)), (dh.stride(0), 1))[:, H:] == 0)


def test_mlp_matches_reference_golden_g6(gpu):
    """Reference MLP (golden G6 from torchrec.model.layer.MLP) through our MLP on
    the GPU: forward and all gradients, bf16 tolerance."""
    from pytorchrec_amd.model.layer import MLP
    gd = golden("g6_mlp.npz")
    n = int(gd["n_layers"])
    units = [gd["W0"].shape[1]] + [gd[f"W{i}"].shape[0] for i in range(n)]
    mlp = MLP(units[0], units[1:], "relu", 0.0).to(gpu)
    lins = [m for m in mlp.modules() if isinstance(m, torch.nn.Linear)]
    with torch.no_grad():
        for i, m in enumerate(lins):
            m.weight.copy_(torch.from_numpy(gd[f"W{i}"]))
            m.bias.copy_(torch.from_numpy(gd[f"b{i}"]))
    x = torch.from_numpy(gd["x"]).to(gpu).requires_grad_()
    y = mlp(x)
    y.backward(torch.from_numpy(gd["dout"]).to(gpu).to(y.dtype))
    # bf16 activations: compare against the golden fp32 values with bf16-level tolerance
    for got, want in [(y.float(), gd["y"]), (x.grad.float(), gd["dx"])] + \
            [(m.weight.grad, gd[f"dW{i}"]) for i, m in enumerate(lins)] + \
            [(m.bias.grad, gd[f"db{i}"]) for i, m in enumerate(lins)]:
        g_ = got.detach().cpu().numpy()
        np.testing.assert_allclose(g_, want, rtol=3e-2, atol=3e-2 * np.abs(want).max())


@pytest.mark.parametrize("net", [False, True])
def test_dcn_cross_forward_backward(gpu, net):
    """net=False: layer by layer (dense.cross); net=True: the whole cross network as
    one autograd node (dense.cross_net, mrec_dcn_cross_bwd_prep)."""
    from pytorchrec_amd import dense as D
    rng = np.random.default_rng(21)
    M, d = 256, 45
    x0 = torch.from_numpy(rng.standard_normal((M, d)).astype(np.float32)).to(torch.bfloat16)
    W = [torch.from_numpy((rng.standard_normal((d, d)) * 0.1).astype(np.float32)) for _ in range(3)]
    b = [torch.from_numpy((rng.standard_normal(d) * 0.1).astype(np.float32)) for _ in range(3)]
    Wg = [w.to(gpu).requires_grad_() for w in W]
    bg = [v.to(gpu).requires_grad_() for v in b]
    x0g = x0.to(gpu).requires_grad_()
    if net:
        x = D.cross_net(x0g, Wg, bg)
    else:
        x = x0g
        for i in range(3):
            x = D.cross(x0g, x, Wg[i], bg[i])
    dout = rng.standard_normal((M, d)).astype(np.float32)
    x.backward(torch.from_numpy(dout).to(gpu).to(x.dtype))
    layers = [(w.numpy(), v.numpy()) for w, v in zip(W, b)]
    x0n = x0.float().numpy()
    xs, zs = ref.dcn_cross_fwd(x0n, layers)
    dx0, grads = ref.dcn_cross_bwd(xs, zs, layers, ref.bf16_round(dout))
    np.testing.assert_allclose(x.detach().float().cpu().numpy(), xs[-1], rtol=0.05,
                               atol=0.05 * np.abs(xs[-1]).max())
    np.testing.assert_allclose(x0g.grad.float().cpu().numpy(), dx0, rtol=0.05,
                               atol=0.05 * np.abs(dx0).max())
    for i in range(3):
        np.testing.assert_allclose(Wg[i].grad.cpu().numpy(), grads[i][0], rtol=0.05,
                                   atol=0.05 * np.abs(grads[i][0]).max())
        np.testing.assert_allclose(bg[i].grad.cpu().numpy(), grads[i][1], rtol=0.05,
                                   atol=0.05 * np.abs(grads[i][1]).max())


def test_deepfm_train_step_matches_oracle_model(gpu):
    """One DeepFM train step on the GPU (fp32 tables, bf16 MLP) vs the oracle's
    reference-path model (fp64) from identical weights: loss and updated tables."""
    import torch.nn as nn
    from oracle.models import RefDeepFM, criteo_batch, sgd_train_step
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    nums = [50, 80, 3, 200, 17, 64]
    F, ND, B = len(nums), 5, 512
    sparse = [CategoricalColumnWithIdentity(n, f"c{f}") for f, n in enumerate(nums)]
    dense = [NumericColumn(f"d{j}") for j in range(ND)]
    lab = CategoricalColumnWithIdentity(2, "label")
    m = DeepFM(sparse, dense, lab, emb_size=16, layers=(64, 32), device=gpu, random_seed=3)
    with torch.no_grad():  # larger init so the MLP contributes visibly
        for p in m.mlp.parameters():
            p.mul_(10)
    r = RefDeepFM(nums, ND, 16, (64, 32), dtype=torch.float64)
    with torch.no_grad():
        for f in range(F):
            r.emb[f].weight.copy_(m.embeddings.table(f).double().cpu())
            r.w1[f].weight.copy_(m.embeddings.first_order(f).double().cpu()[:, None])
        r.dense_w.weight.copy_(m.dense_weight.double().cpu()[None])
        r.global_bias.copy_(m.global_bias.double().cpu())
        ml = [x for x in m.mlp.modules() if isinstance(x, nn.Linear)] + [m.prediction]
        rl = [x for x in r.mlp.modules() if isinstance(x, nn.Linear)] + [r.out]
        for a, b_ in zip(ml, rl):
            b_.weight.copy_(a.weight.double().cpu())
            b_.bias.copy_(a.bias.double().cpu())
    ids, dn, label = criteo_batch(nums, B, n_dense=ND, seed=4)
    data = {c.feature_name: ids[:, f].to(gpu) for f, c in enumerate(sparse)}
    data.update({c.feature_name: dn[:, j].to(gpu) for j, c in enumerate(dense)})
    data["label"] = label.to(gpu)
    lr = 0.5
    before = [r.emb[f].weight.detach().clone() for f in range(F)]
    before_w = [r.w1[f].weight.detach()[:, 0].clone() for f in range(F)]
    m.compile(torch.optim.SGD(m.get_parameters(), lr=lr), torch.nn.BCEWithLogitsLoss(), [], gpu)
    assert m.embeddings.update == "sgd"
    loss = float(m.train_step(data)["loss"])
    ropt = torch.optim.SGD(r.parameters(), lr=lr)
    rloss = float(sgd_train_step(r, ropt, ids, dn.double(), label))
    assert abs(loss - rloss) < 2e-3 * max(1.0, abs(rloss)), (loss, rloss)
    # compare the UPDATES (after - before): bf16 MLP -> a few % relative
    for f in range(F):
        d_got = m.embeddings.table(f).detach().double().cpu() - before[f]
        d_want = r.emb[f].weight.detach() - before[f]
        scale = float(d_want.abs().max()) + 1e-12
        assert float((d_got - d_want).abs().max()) <= 0.05 * scale, f
        dw_got = m.embeddings.first_order(f).detach().double().cpu() - before_w[f]
        dw_want = r.w1[f].weight.detach()[:, 0] - before_w[f]
        assert float((dw_got - dw_want).abs().max()) <= 0.02 * (float(dw_want.abs().max()) + 1e-12)


def test_fused_sgd_linear_matches_torch_sgd(gpu):
    """Plain SGD fused into the weight-gradient GEMM (IModel.compile marks the
    parameters): W -= lr dW, b -= lr db and refreshed bf16 images, against
    torch.optim.SGD applied to the gradients of the unfused path."""
    from pytorchrec_amd import dense as D
    from pytorchrec_amd.model.layer import MLP
    torch.manual_seed(0)
    a = MLP(96, [64, 48], "relu", 0.0).to(gpu)
    b = MLP(96, [64, 48], "relu", 0.0).to(gpu)
    b.load_state_dict(a.state_dict())
    lr = 0.1
    group = {"lr": lr}
    for p in b.parameters():
        p._mrec_sgd_group = group
    x = torch.randn(300, 96, device=gpu).to(torch.bfloat16)
    dout = torch.randn(300, 48, device=gpu).to(torch.bfloat16)
    for _ in range(2):
        a(x).backward(dout)
        with torch.no_grad():
            for p in a.parameters():
                p -= lr * p.grad
                p.grad = None
        b(x).backward(dout)
    for (k, pa), pb in zip(a.state_dict().items(), b.state_dict().values()):
        assert pb.grad is None if hasattr(pb, "grad") else True
        np.testing.assert_allclose(pb.cpu().numpy(), pa.cpu().numpy(), rtol=1e-5, atol=1e-6,
                                   err_msg=k)
    for m in b.modules():
        if isinstance(m, torch.nn.Linear):
            wr, wt = D.weight_images(m.weight)
            wr2, wt2 = D.weight_prep(m.weight)
            assert torch.equal(wr, wr2) and torch.equal(wt, wt2)


def test_colsum_and_fused_update(gpu):
    from pytorchrec_amd import dense as D
    g = torch.Generator().manual_seed(2)
    B, H = 4096, 400
    s = torch.randn(B, generator=g).to(gpu)
    X = D._alloc(B, H, torch.bfloat16, gpu)
    X.copy_(torch.randn(B, H, generator=g).to(torch.bfloat16))
    out, tot = D.colsum(s, X)
    want = (s.double()[:, None] * X.double()).sum(0)
    np.testing.assert_allclose(out.cpu().numpy(), want.cpu().numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(tot.item(), s.double().sum().item(), rtol=1e-5, atol=1e-4)
    out2, tot2 = D.colsum(s, X)
    assert torch.equal(out, out2) and torch.equal(tot, tot2)  # deterministic
    dense = torch.rand(B, 13, generator=g).to(gpu)  # fp32, unaligned rows
    o3, _ = D.colsum(s, dense, want_total=False)
    np.testing.assert_allclose(o3.cpu().numpy(), (s.double()[:, None] * dense.double()).sum(0).cpu().numpy(),
                               rtol=1e-4, atol=1e-3)
    w = torch.randn(13, device=gpu)
    b = torch.randn(1, device=gpu)
    w0, b0 = w.clone(), b.clone()
    D.colsum(s, dense, want_total=True, out=w, total=b, sgd_lr=0.5)
    torch.testing.assert_close(w, w0 - 0.5 * o3, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b, b0 - 0.5 * tot, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("gscale", [1.0, 0.37])
def test_ctr_head_bce_fused_matches_torch(gpu, gscale):
    """Fused Linear(H,1) + BCEWithLogits (mean): loss, logits and every gradient
    against torch fp64 on the same bf16 h (ReLU-masked dh)."""
    from pytorchrec_amd import dense as D
    g = torch.Generator().manual_seed(11)
    B, H = 1000, 400
    hraw = torch.relu(torch.randn(B, H, generator=g)).to(torch.bfloat16)
    h = D._alloc(B, H, torch.bfloat16, gpu)
    h.copy_(hraw)
    setattr(h, D._RELU_OUT, True)
    W = (torch.randn(1, H, generator=g) * 0.05).to(gpu).requires_grad_()
    b = torch.randn(1, generator=g).to(gpu).requires_grad_()
    base = torch.randn(B, generator=g).to(gpu).requires_grad_()
    y = (torch.rand(B, generator=g) < 0.3).float().to(gpu)
    xs = torch.rand(B, 13, generator=g).to(gpu)          # side linear (dense first order)
    ws = (torch.randn(13, generator=g) * 0.1).to(gpu).requires_grad_()
    b2 = torch.randn(1, generator=g).to(gpu).requires_grad_()
    hh = h.detach().clone().requires_grad_()
    setattr(hh, D._RELU_OUT, True)
    loss, z = D.ctr_head_bce(hh, W, b, base, y, xs=xs, ws=ws, b2=b2)
    gl = D.grad_one(gpu) if gscale == 1.0 else torch.tensor(gscale, device=gpu)
    loss.backward(gl)
    Wr = W.detach().double().requires_grad_()
    br = b.detach().double().requires_grad_()
    baser = base.detach().double().requires_grad_()
    hr = hraw.double().to(gpu).requires_grad_()
    wsr = ws.detach().double().requires_grad_()
    b2r = b2.detach().double().requires_grad_()
    zr = baser + hr @ Wr.T.reshape(-1) + br + xs.double() @ wsr + b2r
    lr_ = torch.nn.functional.binary_cross_entropy_with_logits(zr, y.double())
    (lr_ * gscale).backward()
    torch.testing.assert_close(z.double(), zr.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss.double(), lr_.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(W.grad.double(), Wr.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(b.grad.double(), br.grad, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(base.grad.double(), baser.grad, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(ws.grad.double(), wsr.grad, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(b2.grad.double(), b2r.grad, rtol=1e-4, atol=1e-7)
    want_dh = hr.grad * (hr.detach() > 0)
    # one bf16 rounding of dh; a second one when a non-unit loss gradient rescales it
    tol = 2 ** -8 if gscale == 1.0 else 2 ** -7
    torch.testing.assert_close(hh.grad.double(), want_dh, rtol=tol, atol=1e-7)


def test_dcnv2_fused_step_matches_unfused(gpu):
    """DCN-v2 train step with every dense update fused into the backward kernels
    (cross network as one autograd node + multi-GEMM launches) == the same step
    with gradients returned to torch.optim.SGD (up to fp32 fma-vs-mul-add)."""
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.model import DCNv2
    nums = [50, 80, 3, 200]
    sparse = [CategoricalColumnWithIdentity(n, f"c{f}") for f, n in enumerate(nums)]
    dense = [NumericColumn(f"d{j}") for j in range(5)]
    lab = CategoricalColumnWithIdentity(2, "label")
    ms = [DCNv2(sparse, dense, lab, emb_size=16, cross_layers=3, layers=(64, 32), device=gpu,
                random_seed=3) for _ in range(2)]
    with torch.no_grad():
        for p in ms[0].parameters():
            if p.dim() == 2 and p.shape[0] == p.shape[1]:
                p.mul_(20.0)  # cross weights large enough to matter
    ms[1].load_state_dict(ms[0].state_dict())
    for m in ms:
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
    for p in ms[1].parameters():  # force the unfused path on model 1
        if hasattr(p, "_mrec_sgd_group"):
            del p._mrec_sgd_group
    g = torch.Generator().manual_seed(9)
    B = 512
    data = {c.feature_name: torch.randint(0, c.category_num, (B,), generator=g).to(gpu)
            for c in sparse}
    data.update({c.feature_name: torch.rand(B, generator=g).to(gpu) for c in dense})
    data["label"] = (torch.rand(B, generator=g) < 0.3).to(torch.int32).to(gpu)
    for _ in range(2):
        la = float(ms[0].train_step(data)["loss"].detach())
        lb = float(ms[1].train_step(data)["loss"].detach())
        assert abs(la - lb) <= 1e-5 * abs(lb), (la, lb)
    for (k, va), vb in zip(ms[0].state_dict().items(), ms[1].state_dict().values()):
        if "cross" in k or "mlp" in k or "prediction" in k:
            torch.testing.assert_close(va.float(), vb.float(), rtol=1e-4, atol=1e-6, msg=k)
