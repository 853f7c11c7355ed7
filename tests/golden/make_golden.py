"""Generate the golden vectors G1-G8 (+G10-G12) by running the reference itself.

Run IN THE BUILD CONTAINER ONLY (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python tests/golden/make_golden.py

Each fixture is data only (inputs + the reference's outputs) and records the
torch version that produced it (the arithmetic is ATen's).
Shapes are kept small so the fixtures stay a few hundred KB in total; full-size
behaviour is covered by property tests on the GPU.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def _save(name, **arrays):
    arrays["torch_version"] = np.array(torch.__version__)
    np.savez_compressed(os.path.join(OUT, name), **arrays)
    print("wrote", name, {k: getattr(v, "shape", None) for k, v in arrays.items()})


def _bits(t: torch.Tensor) -> np.ndarray:
    assert t.dtype == torch.bfloat16
    return t.contiguous().view(torch.int16).numpy().view(np.uint16)


def main():
    if "torchrec" not in sys.modules:
        try:
            import torchrec  # noqa: F401  (the reference, via PYTHONPATH)
        except ImportError:
            raise SystemExit("run with PYTHONPATH=/root/reference")
    from torchrec.feature_column import (CategoricalColumnWithIdentity, CrossedColumn,
                                         NumericColumn, NormalizationMode)
    from torchrec.model.FunkSVD import FunkSVD
    from torchrec.model.SVDPP import SVDPP
    from torchrec.model.NCF import NCF
    from torchrec.model.SASRec import scaled_dot_product_attention
    from torchrec.model.utils import get_valid_his_index
    from torchrec.model.layer.MLP import MLP
    from torchrec.metric.metrics import get_metric

    torch.set_num_threads(1)

    # ---- G1: nn.Embedding gather on IModel-initialised tables (seed 2020) ------
    rows_u, rows_i, D = 50, 37, 8
    ucol = CategoricalColumnWithIdentity(rows_u, "uid")
    icol = CategoricalColumnWithIdentity(rows_i, "iid")
    lcol = CategoricalColumnWithIdentity(2, "label")
    funk = FunkSVD(uid_column=ucol, iid_column=icol, label_column=lcol, emb_size=D,
                   random_seed=2020)
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, rows_u, (61,), generator=g)
    ids = torch.cat([ids, torch.tensor([0, rows_u - 1, 3, 3, 0, rows_u - 1, 7])])
    table = funk.u_embeddings.weight.detach().clone()
    out = funk.u_embeddings(ids).detach()
    table_bf = table.to(torch.bfloat16)
    out_bf = torch.nn.functional.embedding(ids, table_bf)
    oob_raises = False
    try:
        funk.u_embeddings(torch.tensor([rows_u]))
    except IndexError:
        oob_raises = True
    _save("g1_gather.npz", table=table.numpy(), ids=ids.numpy(), out=out.numpy(),
          table_bf16=_bits(table_bf), out_bf16=_bits(out_bf), oob_raises=np.array(oob_raises))

    # ---- G2: dense grad of nn.Embedding (embedding_dense_backward) -------------
    emb = torch.nn.Embedding(rows_u, D)
    emb.weight.data.copy_(table)
    dy = torch.randn(ids.shape[0], D, generator=g)
    emb(ids).backward(dy)
    _save("g2_dense_grad.npz", ids=ids.numpy(), dy=dy.numpy(), grad=emb.weight.grad.numpy(),
          rows=np.array(rows_u))

    # ---- G3: FunkSVD.forward == FM over {uid, iid} -----------------------------
    B = 64
    batch = {"uid": torch.randint(0, rows_u, (B,), generator=g).int(),
             "iid": torch.randint(0, rows_i, (B,), generator=g).int(),
             "label": torch.randint(0, 2, (B,), generator=g).int()}
    funk.eval()
    with torch.no_grad():
        pred, tgt = funk(batch)
    _save("g3_funksvd.npz", u_table=funk.u_embeddings.weight.detach().numpy(),
          i_table=funk.i_embeddings.weight.detach().numpy(), uid=batch["uid"].numpy(),
          iid=batch["iid"].numpy(), label=batch["label"].numpy(), prediction=pred.numpy(),
          target=tgt.numpy())

    # ---- G10: one IModel.train_step of FunkSVD with dense-grad SGD -------------
    funk2 = FunkSVD(uid_column=ucol, iid_column=icol, label_column=lcol, emb_size=D,
                    random_seed=2020)
    before_u = funk2.u_embeddings.weight.detach().clone()
    before_i = funk2.i_embeddings.weight.detach().clone()
    lr = 0.5
    funk2.compile(optimizer=torch.optim.SGD(funk2.get_parameters(), lr=lr),
                  loss=torch.nn.MSELoss(), metrics=[get_metric("ndcg@10")],
                  device=torch.device("cpu"))
    logs = funk2.train_step(dict(batch))
    _save("g10_funksvd_sgd_step.npz", u_before=before_u.numpy(), i_before=before_i.numpy(),
          u_after=funk2.u_embeddings.weight.detach().numpy(),
          i_after=funk2.i_embeddings.weight.detach().numpy(), uid=batch["uid"].numpy(),
          iid=batch["iid"].numpy(), label=batch["label"].numpy(), lr=np.array(lr),
          loss=np.array(float(logs["loss"])))

    # ---- G4: SVDPP.forward (masked sum/sqrt(len) pooling + biases) -------------
    L = 9
    hcol = CategoricalColumnWithIdentity(rows_i, "iids")
    svdpp = SVDPP(random_seed=2020, uid_column=ucol, iid_column=icol, iids_column=hcol,
                  label_column=lcol, emb_size=D)
    with torch.no_grad():
        svdpp.global_bias.fill_(0.0375)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    his = torch.randint(1, rows_i, (B, L), generator=g)
    his = his * (torch.arange(L)[None, :] < lens[:, None])
    b4 = dict(batch)
    b4["iids"] = his.int()
    svdpp.eval()
    with torch.no_grad():
        pred4, _ = svdpp(b4)
    _save("g4_svdpp.npz", u_table=svdpp.u_embeddings.weight.detach().numpy(),
          i_table=svdpp.i_embeddings.weight.detach().numpy(),
          imp_table=svdpp.implicit_i_embeddings.weight.detach().numpy(),
          ub_table=svdpp.u_bias.weight.detach().numpy(),
          ib_table=svdpp.i_bias.weight.detach().numpy(),
          global_bias=np.array(float(svdpp.global_bias)), uid=batch["uid"].numpy(),
          iid=batch["iid"].numpy(), his=his.numpy(), prediction=pred4.numpy())

    # ---- G5: SASRec masked attention (pins DIN's masked-softmax semantics) -----
    Bq, Lk, E = 16, 12, 8
    q = torch.randn(Bq, 1, E, generator=g)
    k = torch.randn(Bq, Lk, E, generator=g)
    hid = torch.randint(0, 5, (Bq, Lk), generator=g)  # 0 = PAD
    valid = get_valid_his_index(hid)
    mask = (-valid.unsqueeze(1) + 1)  # SASRec.py:95 form: 1 = excluded
    ctx = scaled_dot_product_attention(q, k, k, scale=E ** -0.5, attn_mask=mask)
    _save("g5_sasrec_attn.npz", q=q.numpy(), k=k.numpy(), his_ids=hid.numpy(),
          valid=valid.numpy(), mask=mask.numpy(), scale=np.array(E ** -0.5),
          context=ctx.numpy())

    # ---- G6: reference MLP fwd/bwd (dropout 0) ---------------------------------
    torch.manual_seed(2020)
    units = [45, 32, 32, 16]
    mlp = MLP(input_units=units[0], hidden_units_list=units[1:], activation="relu", dropout=0.0)
    from torchrec.model.IModel import IModel
    mlp.apply(IModel._reset_weights_fn)
    with torch.no_grad():  # larger weights so the ReLU masks are non-trivial
        for m in mlp.modules():
            if isinstance(m, torch.nn.Linear):
                m.weight.mul_(20.0)
                m.bias.mul_(20.0)
    x = torch.randn(16, units[0], generator=g, requires_grad=True)
    y = mlp(x)
    dout = torch.randn(y.shape, generator=g)
    y.backward(dout)
    lin = [m for m in mlp.modules() if isinstance(m, torch.nn.Linear)]
    arrs = {"x": x.detach().numpy(), "y": y.detach().numpy(), "dout": dout.numpy(),
            "dx": x.grad.numpy(), "n_layers": np.array(len(lin))}
    for i, m in enumerate(lin):
        arrs[f"W{i}"] = m.weight.detach().numpy()
        arrs[f"b{i}"] = m.bias.detach().numpy()
        arrs[f"dW{i}"] = m.weight.grad.numpy()
        arrs[f"db{i}"] = m.bias.grad.numpy()
    _save("g6_mlp.npz", **arrs)

    # ---- G7: NCF.forward (embedding concat -> MLP -> Linear) -------------------
    ncf = NCF(random_seed=2020, uid_column=ucol, iid_column=icol, label_column=lcol,
              emb_size=D, layers=[16, 8], dropout=0.0)
    with torch.no_grad():
        for m in ncf.modules():
            if isinstance(m, (torch.nn.Linear, torch.nn.Embedding)):
                m.weight.mul_(30.0)
                if getattr(m, "bias", None) is not None:
                    m.bias.mul_(30.0)
    sample_n = 3
    b7 = {"uid": batch["uid"][:32], "iid": torch.randint(0, rows_i, (32, sample_n), generator=g).int()}
    ncf.eval()
    with torch.no_grad():
        pred7, _ = ncf(b7)
    lin7 = [m for m in ncf.mlp.modules() if isinstance(m, torch.nn.Linear)]
    _save("g7_ncf.npz", uid=b7["uid"].numpy(), iid=b7["iid"].numpy(),
          mf_u=ncf.mf_u_embeddings.weight.detach().numpy(),
          mf_i=ncf.mf_i_embeddings.weight.detach().numpy(),
          mlp_u=ncf.mlp_u_embeddings.weight.detach().numpy(),
          mlp_i=ncf.mlp_i_embeddings.weight.detach().numpy(),
          W0=lin7[0].weight.detach().numpy(), b0=lin7[0].bias.detach().numpy(),
          W1=lin7[1].weight.detach().numpy(), b1=lin7[1].bias.detach().numpy(),
          Wp=ncf.prediction.weight.detach().numpy(), prediction=pred7.numpy())

    # ---- G8: CrossedColumn ids and NumericColumn normalisations ----------------
    c1 = CategoricalColumnWithIdentity(7, "a")
    c2 = CategoricalColumnWithIdentity(5, "b")
    c3 = CategoricalColumnWithIdentity(3, "c")
    cross = CrossedColumn([c1, c2, c3])
    bc = {"a": torch.randint(0, 7, (40,), generator=g).int(),
          "b": torch.randint(0, 5, (40,), generator=g).int(),
          "c": torch.randint(0, 3, (40,), generator=g).int(),
          "x": (torch.rand(40, generator=g) * 10 - 3)}
    num = NumericColumn("x", min_value=-3.0, max_value=7.0, mean_value=2.0, std_value=2.9)
    _save("g8_columns.npz", a=bc["a"].numpy(), b=bc["b"].numpy(), c=bc["c"].numpy(),
          x=bc["x"].numpy(), crossed=cross.get_feature_data(bc).numpy(),
          category_num=np.array(cross.category_num),
          coefficients=np.array(cross.coefficients),
          nop=num.get_feature_data(bc, NormalizationMode.NOP).numpy(),
          max_min=num.get_feature_data(bc, NormalizationMode.MAX_MIN).numpy(),
          z_score=num.get_feature_data(bc, NormalizationMode.Z_SCORE).numpy())

    # ---- G11: FunkSVD sampled (ranking) branch, iid [B, N] ----------------------
    # (FunkSVD.py:56-65: prediction [B, N] = u_b . i_{b,n}, target [B, N] with
    # column 0 = 1); own generator so G1-G10 stay byte-identical
    g11 = torch.Generator().manual_seed(1111)
    n_cand = 5
    b11 = {"uid": torch.randint(0, rows_u, (24,), generator=g11).int(),
           "iid": torch.randint(0, rows_i, (24, n_cand), generator=g11).int()}
    b11["iid"][3, :] = 0  # repeated candidates / row 0 are ordinary rows
    b11["iid"][4, 1:] = b11["iid"][4, 0]
    funk.eval()
    with torch.no_grad():
        pred11, tgt11 = funk(b11)
    _save("g11_funksvd_sampled.npz", u_table=funk.u_embeddings.weight.detach().numpy(),
          i_table=funk.i_embeddings.weight.detach().numpy(), uid=b11["uid"].numpy(),
          iid=b11["iid"].numpy(), prediction=pred11.numpy(), target=tgt11.numpy())


def g12():
    """G12: the reference optimizers' dense steps over an embedding-shaped table
    whose rows get no gradient on some steps (rows still move under Adam's
    momentum): torchrec.optim.AdamW (AdamW.py:21-61; with and without
    correct_bias, weight decay) and get_optimizer("adam") (optimizers.py:9,
    torch.optim.Adam, L2 weight decay).  Pins oracle/ref.py adamw_step / adam_step
    and the fused row-sparse Adam (tests/test_gpu_optim.py)."""
    if "torchrec" not in sys.modules:
        try:
            import torchrec  # noqa: F401
        except ImportError:
            raise SystemExit("run with PYTHONPATH=/root/reference")
    from torchrec.optim.AdamW import AdamW
    from torchrec.optim.optimizers import get_optimizer
    torch.set_num_threads(1)
    g = torch.Generator().manual_seed(1212)
    rows, D, steps = 12, 5, 4
    w0 = torch.randn(rows, D, generator=g) * 0.1
    grads = torch.randn(steps, rows, D, generator=g) * 0.5
    mask = torch.rand(steps, rows, generator=g) < 0.5  # rows looked up at each step
    grads = grads * mask[..., None]
    out = {"w0": w0.numpy(), "grads": grads.numpy(), "mask": mask.numpy()}
    configs = {"adamw": lambda p: AdamW([p], lr=0.05, betas=(0.9, 0.999), eps=1e-6,
                                        weight_decay=0.1, correct_bias=True),
               "adamw_nobc": lambda p: AdamW([p], lr=0.05, eps=1e-6, correct_bias=False),
               "adam": lambda p: get_optimizer("adam")([p], lr=0.05, betas=(0.8, 0.99),
                                                       eps=1e-8, weight_decay=0.05)}
    import warnings
    for name, make in configs.items():
        p = torch.nn.Parameter(w0.clone())
        opt = make(p)
        traj = []
        for s in range(steps):
            p.grad = grads[s].clone()
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")  # the reference's deprecated add_(alpha, t)
                opt.step()
            traj.append(p.detach().clone().numpy())
        out[name] = np.stack(traj)
    _save("g12_optimizers.npz", **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["g12"]:
        g12()
    else:
        main()
        g12()
