"""The fused MLP tower (mrec_tower_fwd_bwd: MLP forward + Linear(N_L, 1) head +
BCE + the whole input-gradient backward in one launch) against

  * the fp64 oracle (ref.mlp_fwd / mlp_bwd / bce_with_logits) on the same bf16
    operands: bf16 activations and gradients (<= 2^-8 per rounding) through up to
    4 layers -> 3 % of each tensor's magnitude;
  * the layered path (one mrec_gemm per layer + mrec_ctr_head_fwd), which rounds
    at exactly the same points: only fp32 accumulation order differs, so the
    outputs agree to a couple of bf16 ulps and the loss to 1e-6;
  * whole train steps of DeepFM / DCN-v2 / DIN with the tower on vs off.

Shapes cover the C2 tower (429 -> 400^3), widths that are not multiples of
16 / 32, 1..4 layers and batches that are not multiples of the 16-row block.
"""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _mlp(widths, gpu, seed, bias_mu=0.0):
    from pytorchrec_amd.model.layer import MLP
    torch.manual_seed(seed)
    m = MLP(widths[0], list(widths[1:]), "relu", 0.0).to(gpu)
    head = torch.nn.Linear(widths[-1], 1).to(gpu)
    with torch.no_grad():
        for lin in [d.linear for d in m.mlp]:
            lin.weight.normal_(0, 1.0 / np.sqrt(lin.in_features))
            lin.bias.normal_(bias_mu, 0.1)
        head.weight.normal_(0, 1.0 / np.sqrt(widths[-1]))
        head.bias.fill_(0.05)
    return m, head


def _x0(B, K, gpu, seed):
    from pytorchrec_amd import dense as D
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(B, D._r8(K), dtype=torch.bfloat16, device=gpu)
    x[:, :K] = torch.randn(B, K, generator=g).to(torch.bfloat16).to(gpu)
    return x[:, :K]


def _run_tower(x0, mlp, head, base, y, xs=None, ws=None, b2=None):
    from pytorchrec_amd import dense as D
    xg = x0.detach().requires_grad_()
    bg = base.detach().requires_grad_() if base is not None else None
    assert D.tower_supported(xg, mlp, head, xs)
    loss = D.tower_bce(xg, mlp, head, bg, y, xs=xs, ws=ws, b2=b2)
    loss.backward()
    return loss, xg.grad, (bg.grad if bg is not None else None)


@pytest.mark.parametrize("widths,B", [((429, 400, 400, 400), 4096), ((45, 70, 33), 1000),
                                      ((32, 200, 80), 513), ((100, 512), 16),
                                      ((16, 64, 48, 32, 17), 77)])
def test_tower_matches_fp64_oracle_and_layered_path(gpu, widths, B):
    """Tight bar: the layered path (same rounding points) — loss within 1e-6, every
    gradient within 0.1 % of its magnitude on average and 99.9 % of the elements
    within 1 %.  Against
    fp64 the bar is what bf16 gradients allow: each backward layer sums ~N terms of
    random sign (|sum| ~ sum|terms| / sqrt(N)), so the 2^-9 rounding of every
    stored gradient is amplified ~sqrt(N) per layer, and the odd near-zero ReLU
    mask flips: 8 % in L2 after three 400-wide layers."""
    from pytorchrec_amd import dense as D
    l2_bar = 8e-2
    mlp, head = _mlp(widths, gpu, seed=B)
    x0 = _x0(B, widths[0], gpu, seed=B + 1)
    g = torch.Generator().manual_seed(B + 2)
    y = (torch.rand(B, generator=g) < 0.3).float().to(gpu)
    base = (torch.randn(B, generator=g) * 0.5).to(gpu)
    ns = 5
    xs = torch.rand(B, ns, generator=g).to(gpu)
    ws = (torch.randn(ns, generator=g) * 0.1).to(gpu).requires_grad_()
    b2 = torch.full((1,), 0.02, device=gpu).requires_grad_()
    loss, dx0, dbase = _run_tower(x0, mlp, head, base, y, xs, ws, b2)
    lins = [d.linear for d in mlp.mlp]
    grads = [(l.weight.grad.clone(), l.bias.grad.clone()) for l in lins]
    hgrads = (head.weight.grad.clone(), head.bias.grad.clone(), ws.grad.clone(), b2.grad.clone())

    # --- the layered path: identical rounding points ----------------------------
    for p in list(mlp.parameters()) + list(head.parameters()) + [ws, b2]:
        p.grad = None
    xg = x0.detach().requires_grad_()
    bg = base.detach().requires_grad_()
    loss2, _ = D.ctr_head_bce(mlp(xg), head.weight, head.bias, bg, y, xs=xs, ws=ws, b2=b2)
    loss2.backward()
    assert abs(float(loss) - float(loss2)) <= 1e-6 * abs(float(loss2)) + 1e-7
    for got, want, name in [(dx0, xg.grad, "dx0"), (dbase, bg.grad, "dz")] + \
            [(grads[l][0], lins[l].weight.grad, f"dW{l}") for l in range(len(lins))] + \
            [(grads[l][1], lins[l].bias.grad, f"db{l}") for l in range(len(lins))]:
        got, want = got.double().cpu(), want.double().cpu()
        mag = float(want.abs().max()) + 1e-30
        err = (got - want).abs()
        # a 1-ulp difference in an activation that sits at a ReLU's zero can flip
        # that unit's mask: rare elements may differ by a whole term
        assert float(err.mean()) <= 1e-3 * mag, (name, float(err.mean()) / mag)
        assert float((err > 1e-2 * mag).double().mean()) <= 1e-3, name

    # --- fp64 oracle on the same bf16 weights / inputs --------------------------
    layers = [(ref.bf16_round(l.weight.detach().cpu().numpy()), l.bias.detach().cpu().numpy())
              for l in lins]
    xn = x0.detach().float().cpu().numpy()
    acts = ref.mlp_fwd(xn, layers)
    hw = head.weight.detach().cpu().numpy().reshape(-1)
    z = acts[-1] @ hw + float(head.bias) + base.cpu().numpy() + xs.cpu().numpy() @ ws.detach().cpu().numpy() + float(b2)
    want_loss, dz = ref.bce_with_logits(z, y.cpu().numpy())
    assert abs(float(loss) - want_loss) <= 3e-3 * abs(want_loss), (float(loss), want_loss)
    np.testing.assert_allclose(dbase.cpu().numpy(), dz, rtol=3e-2, atol=3e-2 * np.abs(dz).max())
    dx_ref, lgr = ref.mlp_bwd(acts, layers, dz[:, None] * hw[None, :])

    def close(got, want, name):
        got = got.detach().double().cpu().numpy().reshape(want.shape)
        l2 = np.linalg.norm(got - want) / (np.linalg.norm(want) + 1e-30)
        assert l2 <= l2_bar, (name, l2)

    close(dx0, dx_ref, "dx0")
    for l, ((dW, db), (wW, wb)) in enumerate(zip(grads, lgr)):
        close(dW, wW, f"dW{l}")
        close(db, wb, f"db{l}")
    close(hgrads[0].reshape(-1), acts[-1].T @ dz, "dW_head")
    close(hgrads[1], np.array([dz.sum()]), "db_head")
    close(hgrads[2], xs.cpu().numpy().T @ dz, "dws")


def test_tower_images_follow_fused_sgd_and_torch_updates(gpu):
    """Fused SGD rewrites the tower images in the weight-gradient reduction: a
    second step must see the updated weights (== recomputing the images from the
    fp32 masters), and a torch in-place update (version bump) re-preps them."""
    from pytorchrec_amd import dense as D
    mlp, head = _mlp((64, 48, 32), gpu, seed=3)
    lins = [d.linear for d in mlp.mlp]
    for p in list(mlp.parameters()) + list(head.parameters()):
        p._mrec_sgd_group = {"lr": 0.1}
    x0 = _x0(256, 64, gpu, seed=4)
    y = (torch.rand(256, generator=torch.Generator().manual_seed(5)) < 0.5).float().to(gpu)
    for _ in range(2):
        loss = D.tower_bce(x0.detach().requires_grad_(), mlp, head, None, y)
        loss.backward(D.grad_one(gpu))
        D.flush_pending()
    torch.cuda.synchronize()
    for l in lins:
        pf, pb = D.cached_images(l.weight, "tower")
        fresh_f = torch.zeros_like(pf)
        fresh_b = torch.zeros_like(pb)
        from pytorchrec_amd import _mrec
        W = l.weight.detach()
        _mrec.call("mrec_tower_weight_prep", W.data_ptr(), W.shape[0], W.shape[1], W.stride(0),
                   fresh_f.data_ptr(), fresh_b.data_ptr(), _mrec.stream_handle())
        assert torch.equal(pf, fresh_f) and torch.equal(pb, fresh_b)
    with torch.no_grad():
        lins[0].weight.mul_(0.5)  # torch update: version bump
    assert D.cached_images(lins[0].weight, "tower") is None
    for p in list(mlp.parameters()) + list(head.parameters()):
        del p._mrec_sgd_group


@pytest.mark.parametrize("model", ["deepfm", "dcnv2", "din"])
def test_train_steps_tower_on_vs_off(gpu, model):
    """Three train steps of each CTR model with the tower and with the layered
    path from the same weights: same losses (1e-5) and parameters within bf16
    accumulation-order differences."""
    import bench
    from pytorchrec_amd import dense as D
    from pytorchrec_amd.loss import BCEWithLogitsLoss

    class A:
        batch, lr, rows_per_table, zipf, shard_cap = 1000, 0.05, 5000, 0.0, None
    build = {"deepfm": bench.build_deepfm, "dcnv2": bench.build_dcnv2, "din": bench.build_din}[model]
    runs = []
    for tower in (True, False):
        D.TOWER = tower
        try:
            m = build(A, gpu)[0]
            m.compile(torch.optim.SGD(m.get_parameters(), lr=A.lr), BCEWithLogitsLoss(), [], gpu)
            if model == "din":
                data = bench.din_batch(A, 0, gpu)
            else:
                sparse = [c for c in m.sparse_columns]
                buf = bench.make_batch_buffer(A, sparse, 0, gpu)
                data = bench.batch_views(buf, A, sparse, m.dense_columns, m.label_column)
            losses = [float(m.train_step(data)["loss"].detach()) for _ in range(3)]
            runs.append((losses, {k: v.detach().float().cpu() for k, v in m.state_dict().items()}))
        finally:
            D.TOWER = True
    (la, sa), (lb, sb) = runs
    np.testing.assert_allclose(la, lb, rtol=1e-5)
    for k in sa:
        d = (sa[k] - sb[k]).abs().max().item()
        scale = sb[k].abs().max().item() + 1e-12
        assert d <= 2e-2 * scale, (k, d / scale)


@pytest.mark.parametrize("widths,B", [((128, 80, 40), 3200), ((45, 70, 33), 1000),
                                      ((128, 80, 40), 24000)])
def test_score_tower_matches_layered_path_and_fp64(gpu, widths, B):
    """The score tower (DIN's attention unit: MREC_TOWER_FORWARD scores, then a
    MREC_TOWER_GIVEN_DZ backward that recomputes the forward in LDS) against the
    layered path (one GEMM per layer + Linear(h, 1): the same bf16 rounding points)
    with the bar of the BCE tower's test, and against the fp64 oracle on the same
    bf16 weights / inputs (l2 within 8e-2).  The 24,000-row case runs
    mrec_tower_dw with many K slices."""
    from pytorchrec_amd import dense as D
    mlp, head = _mlp(widths, gpu, seed=B + 7)
    x0 = _x0(B, widths[0], gpu, seed=B + 8)
    g = torch.Generator().manual_seed(B + 9)
    ds = (torch.randn(B, 1, generator=g) * 1e-3).to(gpu)
    lins = [d.linear for d in mlp.mlp]
    params = list(mlp.parameters()) + list(head.parameters())

    xg = x0.detach().requires_grad_()
    assert D.tower_supported(xg, mlp, head)
    s = D.score_tower(xg, mlp, head).reshape(-1, 1)
    s.backward(ds)
    got = {"s": s.detach(), "dx0": xg.grad}
    for i, l in enumerate(lins):
        got[f"dW{i}"], got[f"db{i}"] = l.weight.grad.clone(), l.bias.grad.clone()
    got["dW_head"], got["db_head"] = head.weight.grad.clone(), head.bias.grad.clone()

    for p in params:
        p.grad = None
    xl = x0.detach().requires_grad_()
    sl = D.linear(mlp(xl), head.weight, head.bias, out_dtype=torch.float32)
    sl.backward(ds)
    want = {"s": sl.detach(), "dx0": xl.grad}
    for i, l in enumerate(lins):
        want[f"dW{i}"], want[f"db{i}"] = l.weight.grad, l.bias.grad
    want["dW_head"], want["db_head"] = head.weight.grad, head.bias.grad
    # the layered head rounds dh_L = ds w at a different point (its Linear(h, 1)
    # backward), so sums with heavy cancellation (the bias gradients) differ by
    # ~2^-9 of their magnitude: a 4e-3 mean bar here, the tight bar elsewhere
    for name in want:
        a, b = got[name].double().cpu(), want[name].double().cpu().reshape(got[name].shape)
        mag = float(b.abs().max()) + 1e-30
        err = (a - b).abs()
        assert float(err.mean()) <= 4e-3 * mag, (name, float(err.mean()) / mag)
        assert float((err > 2e-2 * mag).double().mean()) <= 1e-3, name

    layers = [(ref.bf16_round(l.weight.detach().cpu().numpy()), l.bias.detach().cpu().numpy())
              for l in lins]
    acts = ref.mlp_fwd(x0.detach().float().cpu().numpy(), layers)
    hw = head.weight.detach().cpu().numpy().reshape(-1)
    z = acts[-1] @ hw + float(head.bias)
    dz = ds.cpu().numpy().reshape(-1).astype(np.float64)
    dx_ref, lgr = ref.mlp_bwd(acts, layers, dz[:, None] * hw[None, :])

    def close(a, w, name):
        a = a.detach().double().cpu().numpy().reshape(w.shape)
        l2 = np.linalg.norm(a - w) / (np.linalg.norm(w) + 1e-30)
        assert l2 <= 8e-2, (name, l2)

    close(got["s"], z, "s")
    close(got["dx0"], dx_ref, "dx0")
    for l, (wW, wb) in enumerate(lgr):
        close(got[f"dW{l}"], wW, f"dW{l}")
        close(got[f"db{l}"], wb, f"db{l}")
    close(got["dW_head"].reshape(-1), acts[-1].T @ dz, "dW_head")
    close(got["db_head"], np.array([dz.sum()]), "db_head")


@pytest.mark.parametrize("d,mlp_w,C,B", [(429, (400, 400), 3, 4096), (45, (70, 33), 2, 1000),
                                         (100, (64,), 1, 513), (16, (48, 32, 17), 3, 600)])
def test_cross_tower_matches_layered_path_and_fp64(gpu, d, mlp_w, C, B):
    """DCN-v2 cross layers inside the tower launch (mrec_tower_args.n_cross: x_{c+1} =
    x0 * (x_c W_c^T + b_c) + x_c on the x0 block, z_c kept on chip, the cross dW
    from the tower's k-fragment images in the same mrec_tower_dw launch) against

      * the layered path (dense.cross_net: one mrec_gemm per layer + the
        mrec_dcn_cross_bwd_prep elementwise stage, then the MLP tower): the same
        bf16 rounding points except dx0, which the fused path rounds once (fp32
        sum of G_0 and every G_{c+1} z_c) -- loss within 1e-6, every gradient within
        0.1 % of its magnitude on average, 99.9 % of the elements within 1 %
        (dx0: 0.3 % / 3 %, bias gradients 0.4 % / 4 %), the loss within 1e-5;
      * the fp64 oracle (ref.dcn_cross_fwd / _bwd + ref.mlp_fwd / _bwd) on the same
        bf16 x0 and bf16-rounded weights: l2 within 8e-2, as the MLP tower's test."""
    from pytorchrec_amd import dense as D
    widths = (d,) + tuple(mlp_w)
    mlp, head = _mlp(widths, gpu, seed=B + C)
    torch.manual_seed(B + 11)
    cross = [torch.nn.Linear(d, d).to(gpu) for _ in range(C)]
    with torch.no_grad():
        for c in cross:
            c.weight.normal_(0, 1.0 / np.sqrt(d))
            c.bias.normal_(0, 0.1)
    x0 = _x0(B, d, gpu, seed=B + 12)
    g = torch.Generator().manual_seed(B + 13)
    y = (torch.rand(B, generator=g) < 0.3).float().to(gpu)
    lins = [l.linear for l in mlp.mlp]
    params = list(mlp.parameters()) + list(head.parameters()) + [p for c in cross for p in c.parameters()]

    xg = x0.detach().requires_grad_()
    assert D.tower_supported(xg, mlp, head, cross=cross)
    loss = D.tower_bce(xg, mlp, head, None, y, cross=cross)
    loss.backward()
    got = {"dx0": xg.grad.clone()}
    for i, l in enumerate(cross + lins):
        got[f"dW{i}"], got[f"db{i}"] = l.weight.grad.clone(), l.bias.grad.clone()
    got["dW_head"], got["db_head"] = head.weight.grad.clone(), head.bias.grad.clone()

    for p in params:
        p.grad = None
    xl = x0.detach().requires_grad_()
    x = D.cross_net(xl, [c.weight for c in cross], [c.bias for c in cross])
    loss2, _ = D.ctr_head_bce(mlp(x), head.weight, head.bias, None, y)
    loss2.backward()
    # the k steps of a layer are summed in a per-workgroup rotated order in the tower
    # (the GEMM's is fixed): a 1-ulp flip of an x_c element feeds every later layer
    # through both the product and the residual, so the loss bar is 1e-5 here
    assert abs(float(loss) - float(loss2)) <= 1e-5 * abs(float(loss2)) + 1e-7
    want = {"dx0": xl.grad}
    for i, l in enumerate(cross + lins):
        want[f"dW{i}"], want[f"db{i}"] = l.weight.grad, l.bias.grad
    want["dW_head"], want["db_head"] = head.weight.grad, head.bias.grad
    for name in want:
        a, b = got[name].double().cpu(), want[name].double().cpu().reshape(got[name].shape)
        mag = float(b.abs().max()) + 1e-30
        err = (a - b).abs()
        # dx0 is rounded once here (three times on the layered path); the bias
        # gradients sum B terms with heavy cancellation, so a few 1-ulp flips of
        # dz (the rotated k order) move them by ~2^-9 of their magnitude (the score
        # tower's bar)
        k = 3.0 if name == "dx0" else (4.0 if name.startswith("db") else 1.0)
        assert float(err.mean()) <= k * 1e-3 * mag, (name, float(err.mean()) / mag)
        assert float((err > k * 1e-2 * mag).double().mean()) <= 1e-3, name

    clay = [(ref.bf16_round(c.weight.detach().cpu().numpy()), c.bias.detach().cpu().numpy())
            for c in cross]
    layers = [(ref.bf16_round(l.weight.detach().cpu().numpy()), l.bias.detach().cpu().numpy())
              for l in lins]
    xs, zs = ref.dcn_cross_fwd(x0.detach().float().cpu().numpy(), clay)
    acts = ref.mlp_fwd(xs[-1], layers)
    hw = head.weight.detach().cpu().numpy().reshape(-1)
    z = acts[-1] @ hw + float(head.bias)
    want_loss, dz = ref.bce_with_logits(z, y.cpu().numpy())
    assert abs(float(loss) - want_loss) <= 3e-3 * abs(want_loss), (float(loss), want_loss)
    dxc, lgr = ref.mlp_bwd(acts, layers, dz[:, None] * hw[None, :])
    dx0, cgr = ref.dcn_cross_bwd(xs, zs, clay, dxc)

    def close(a, w, name):
        a = a.detach().double().cpu().numpy().reshape(w.shape)
        l2 = np.linalg.norm(a - w) / (np.linalg.norm(w) + 1e-30)
        assert l2 <= 8e-2, (name, l2)

    close(got["dx0"], dx0, "dx0")
    for i, (wW, wb) in enumerate(cgr + lgr):
        close(got[f"dW{i}"], wW, f"dW{i}")
        close(got[f"db{i}"], wb, f"db{i}")
    close(got["dW_head"].reshape(-1), acts[-1].T @ dz, "dW_head")
