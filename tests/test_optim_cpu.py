"""Optimizers on the CPU: the oracle's dense restatements (oracle/ref.py) and the
mirrored ``pytorchrec_amd.optim`` classes against golden G12, produced by the
reference's own AdamW (torchrec/optim/AdamW.py:21-61) and get_optimizer("adam")
(optimizers.py:9) stepping an embedding-shaped table with rows that get no
gradient on some steps (tests/golden/make_golden.py g12)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref


def _oracle_traj(name, g):
    w0, grads = g["w0"].astype(np.float64), g["grads"].astype(np.float64)
    p, m, v = w0.copy(), np.zeros_like(w0), np.zeros_like(w0)
    out = []
    for s in range(grads.shape[0]):
        if name == "adamw":
            ref.adamw_step(p, grads[s], m, v, s + 1, 0.05, (0.9, 0.999), 1e-6, 0.1, True)
        elif name == "adamw_nobc":
            ref.adamw_step(p, grads[s], m, v, s + 1, 0.05, (0.9, 0.999), 1e-6, 0.0, False)
        else:
            ref.adam_step(p, grads[s], m, v, s + 1, 0.05, (0.8, 0.99), 1e-8, 0.05)
        out.append(p.copy())
    return np.stack(out)


@pytest.mark.parametrize("name", ["adamw", "adamw_nobc", "adam"])
def test_oracle_optimizers_match_reference_g12(name):
    g = golden("g12_optimizers.npz")
    np.testing.assert_allclose(_oracle_traj(name, g), g[name], rtol=2e-6, atol=1e-7)


def test_mirrored_adamw_matches_reference_g12():
    from pytorchrec_amd.optim import AdamW
    g = golden("g12_optimizers.npz")
    for name, kw in [("adamw", dict(lr=0.05, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.1)),
                     ("adamw_nobc", dict(lr=0.05, eps=1e-6, correct_bias=False))]:
        p = torch.nn.Parameter(torch.from_numpy(g["w0"].copy()))
        opt = AdamW([p], **kw)
        for s in range(g["grads"].shape[0]):
            p.grad = torch.from_numpy(g["grads"][s].copy())
            opt.step()
            np.testing.assert_allclose(p.detach().numpy(), g[name][s], rtol=1e-6, atol=1e-8)


def test_rowwise_adagrad_matches_oracle():
    from pytorchrec_amd.optim import RowWiseAdagrad
    rng = np.random.default_rng(0)
    w0 = rng.standard_normal((9, 6)).astype(np.float32)
    p = torch.nn.Parameter(torch.from_numpy(w0.copy()))
    opt = RowWiseAdagrad([p], lr=0.1, eps=1e-10)
    want, s = w0.astype(np.float64), np.zeros(9)
    for _ in range(4):
        gr = rng.standard_normal((9, 6)).astype(np.float32) * (rng.random((9, 1)) < 0.6)
        p.grad = torch.from_numpy(gr)
        opt.step()
        ref.rowwise_adagrad_step(want, gr.astype(np.float64), s, 0.1, 1e-10)
    np.testing.assert_allclose(p.detach().numpy(), want, rtol=1e-5, atol=1e-7)


def test_optimizer_registry_and_fused_spec():
    from pytorchrec_amd.optim import AdamW, RowWiseAdagrad, fused_spec, get_optimizer
    assert get_optimizer("sgd") is torch.optim.SGD and get_optimizer("adam") is torch.optim.Adam
    assert get_optimizer("adamw") is AdamW
    with pytest.raises(ValueError):
        get_optimizer("lamb")
    p = [torch.nn.Parameter(torch.zeros(3))]
    spec = lambda o: fused_spec(o, o.param_groups[0])  # noqa: E731
    assert spec(torch.optim.Adagrad(p, lr=0.1))["kind"] == "adagrad"
    assert spec(torch.optim.Adagrad(p, lr=0.1, weight_decay=0.1)) is None  # rows would decay
    assert spec(RowWiseAdagrad(p))["kind"] == "rowwise_adagrad"
    a = spec(AdamW(p, weight_decay=0.1))
    assert a["kind"] == "adam" and a["decoupled"] and a["bias_correction"]
    b = spec(torch.optim.Adam(p, weight_decay=0.2))
    assert b["kind"] == "adam" and not b["decoupled"] and b["weight_decay"] == 0.2
    assert spec(torch.optim.Adam(p, amsgrad=True)) is None
    assert spec(torch.optim.AdamW(p)) is None  # torch's AdamW orders its decay differently
    # torch Adam(decoupled_weight_decay=True) decays before the moment update: dense grad
    assert spec(torch.optim.Adam(p, weight_decay=0.1, decoupled_weight_decay=True)) is None
    c = spec(torch.optim.Adam(p, decoupled_weight_decay=True))  # no decay: plain Adam
    assert c["kind"] == "adam" and c["weight_decay"] == 0.0
