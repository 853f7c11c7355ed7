"""DIN target attention on the GPU (config C4): the attention-unit input builder,
masked-softmax pooling and their fused backward kernels, against an fp64 torch
restatement of the same block (and the numpy oracle for the forward), plus a DIN
train step end to end.  Tolerances: bf16 activations (<= 2^-8 relative each
rounding) through two bf16 MFMA layers -> 3e-2 relative to the magnitude."""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _block(gpu, B=64, L=50, E=32, seed=0):
    from pytorchrec_amd.model.layer import MLP
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    att = MLP(4 * E, [80, 40], "relu", 0.0).to(gpu)
    out = torch.nn.Linear(40, 1).to(gpu)
    with torch.no_grad():
        for p in list(att.parameters()) + list(out.parameters()):
            p.normal_(0, 0.2, generator=None)
    q = torch.randn(B, E, generator=g).to(torch.bfloat16).to(gpu)
    k = torch.randn(B * L, E, generator=g).to(torch.bfloat16).to(gpu)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    his = torch.randint(1, 1000, (B, L), generator=g, dtype=torch.int32)
    his[torch.arange(L)[None, :] >= lens[:, None]] = 0
    return att, out, q, k, his.to(gpu)


def _ref_block(att, out, q, k, his, L):
    """fp64 torch: same math as dense.din_attention on the bf16 inputs."""
    lins = [m for m in att.modules() if isinstance(m, torch.nn.Linear)]
    B, E = q.shape
    qd = q.double().detach().cpu().requires_grad_()
    kd = k.double().detach().cpu().reshape(B, L, E).requires_grad_()
    Ws = [(m.weight.detach().double().cpu(), m.bias.detach().double().cpu()) for m in lins]
    qb = qd[:, None, :].expand(B, L, E)
    x = torch.cat([qb, kd, qb - kd, qb * kd], -1).reshape(B * L, 4 * E)
    for W, b in Ws:
        x = torch.relu(x @ W.T + b)
    s = (x @ out.weight.detach().double().cpu().T + out.bias.detach().double().cpu()).reshape(B, L)
    valid = his.cpu() > 0
    valid[:, 0] = True
    a = torch.softmax(s.masked_fill(~valid, float("-inf")), -1)
    u = (a[..., None] * kd).sum(1)
    return qd, kd, torch.cat([qd, u], -1)


def test_din_forward_matches_oracle_and_torch(gpu):
    from pytorchrec_amd import dense as D
    att, out, q, k, his = _block(gpu)
    B, E = q.shape
    L = his.shape[1]
    with torch.no_grad():
        top = D.din_attention_top(q, k, his, att, out)
    assert torch.equal(top[:, :E], q)  # the concat is exact
    _, _, want = _ref_block(att, out, q, k, his, L)
    got = top.double().cpu()
    mag = want.abs().max().item()
    np.testing.assert_allclose(got.numpy(), want.detach().numpy(), rtol=3e-2, atol=3e-2 * mag)
    # the numpy oracle (fp64) agrees on the pooled vector
    lins = [m for m in att.modules() if isinstance(m, torch.nn.Linear)]
    layers = [(m.weight.detach().double().cpu().numpy(), m.bias.detach().double().cpu().numpy())
              for m in lins]
    u, a, s = ref.din_attention_pool(q.double().cpu().numpy(),
                                     k.double().cpu().numpy().reshape(B, L, E),
                                     ref.valid_his_index(his.cpu().numpy()), layers,
                                     (out.weight.detach().double().cpu().numpy(),
                                      out.bias.detach().double().cpu().numpy()))
    np.testing.assert_allclose(got[:, E:].numpy(), u, rtol=3e-2, atol=3e-2 * np.abs(u).max())


def test_din_rows_path_equals_split_path_bitwise(gpu):
    """din_attention_top_rows (the model's path: one bf16 gradient of the gathered
    rows from mrec_din_feat_bwd_rows) == din_attention_top on the q / k slices with
    autograd casting dq / dk to bf16: same output bits, same gradient bits."""
    from pytorchrec_amd import dense as D
    att, out, q, k, his = _block(gpu, seed=5)
    B, E = q.shape
    rows = torch.cat([q, k]).detach().clone().requires_grad_()
    top_r = D.din_attention_top_rows(rows, B, his, att, out)
    g = torch.Generator().manual_seed(4)
    dtop = torch.randn(B, 2 * E, generator=g).to(gpu).to(top_r.dtype)
    top_r.backward(dtop)
    qg = q.detach().clone().requires_grad_()
    kg = k.detach().clone().requires_grad_()
    top_s = D.din_attention_top(qg, kg, his, att, out)
    top_s.backward(dtop)
    assert torch.equal(top_r, top_s)
    assert rows.grad.dtype == torch.bfloat16
    assert torch.equal(rows.grad[:B], qg.grad.to(torch.bfloat16))
    assert torch.equal(rows.grad[B:], kg.grad.to(torch.bfloat16))


def test_din_backward_matches_torch(gpu):
    from pytorchrec_amd import dense as D
    att, out, q, k, his = _block(gpu, seed=3)
    B, E = q.shape
    L = his.shape[1]
    qg = q.detach().clone().requires_grad_()
    kg = k.detach().clone().requires_grad_()
    top = D.din_attention_top(qg, kg, his, att, out)
    g = torch.Generator().manual_seed(9)
    dtop = torch.randn(B, 2 * E, generator=g)
    top.backward(dtop.to(gpu).to(top.dtype))
    qd, kd, want = _ref_block(att, out, q, k, his, L)
    want.backward(dtop.double().to(torch.bfloat16).double())
    for name, got, ref_ in [("dq", qg.grad, qd.grad), ("dk", kg.grad.reshape(B, L, E), kd.grad)]:
        gg = got.double().cpu()
        assert not torch.isnan(gg).any(), (name, torch.isnan(gg).nonzero()[:8].tolist())
        assert not torch.isnan(ref_).any(), (name, "ref", torch.isnan(ref_).nonzero()[:8].tolist())
        mag = ref_.abs().max().item()
        np.testing.assert_allclose(gg.numpy(), ref_.numpy(), rtol=5e-2, atol=5e-2 * mag)
    # padded history positions get no gradient through the pooling weights
    pad = (his.cpu() == 0)
    pad[:, 0] = False
    dk = kg.grad.reshape(B, L, E).cpu()
    ref_dk = kd.grad
    assert torch.allclose(dk[pad].double(), ref_dk[pad], atol=5e-2 * ref_dk.abs().max().item())


def test_din_train_step_runs_and_learns(gpu):
    import bench
    from pytorchrec_amd.loss import BCEWithLogitsLoss

    class A:
        batch, lr = 512, 0.05
    model, _, _, _ = bench.build_din(A, gpu)
    model.compile(torch.optim.SGD(model.get_parameters(), lr=A.lr), BCEWithLogitsLoss(), [], gpu)
    data = bench.din_batch(A, 0, gpu)
    w0 = model.embeddings.weight.detach().clone()
    losses = [float(model.train_step(data)["loss"].detach()) for _ in range(5)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
    touched = torch.cat([data["iid"], data["pos_his"].reshape(-1)]).unique().long()
    assert not torch.equal(model.embeddings.weight[touched], w0[touched])
