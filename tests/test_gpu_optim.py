"""Fused row-sparse optimizers of the embedding bank (include/mrec.h
MREC_BWD_ADAGRAD / _ROWWISE_ADAGRAD / _ADAM) against the dense optimizers the
reference steps over whole tables (torchrec/optim/AdamW.py:21-61,
optimizers.py:7-20 -> torch.optim.Adam / Adagrad), restated in fp64 by
oracle/ref.py.

Bars: fp32 banks within 1e-5 relative (+ 1e-6 absolute: an Adam step is ~lr and
its fp32 state rounds at ~1e-7 of it per step) of the fp64 dense optimizer after
several steps, including rows left untouched for several steps
(dense Adam still moves them: the fused Adam catches them up on their next lookup
or at flush_optimizer); bf16 banks within one bf16 rounding per step.
"""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _bank(rows, F, D, has_w, dtype, init):
    from pytorchrec_amd import _mrec
    from pytorchrec_amd.embedding import EmbeddingBank
    assert _mrec.available(), "libmrec.so must be built and loadable on the GPU box"
    b = EmbeddingBank([rows] * F, D, with_first_order=has_w, dtype=dtype, device="cuda")
    with torch.no_grad():
        b.weight.zero_()
        for f in range(F):
            o = b.row_offset[f]
            b.weight[o:o + rows, :D + (1 if has_w else 0)] = torch.from_numpy(init[f]).to(
                "cuda", dtype)
    return b


def _table(bank, rows, F, D, has_w):
    w = bank.weight.detach().float().cpu().numpy()
    n = D + (1 if has_w else 0)
    return [w[bank.row_offset[f]:bank.row_offset[f] + rows, :n].astype(np.float64)
            for f in range(F)]


def _ids_schedule(rng, rows, B, steps):
    """Per step, ids of each table: even steps draw from the first half of the
    rows, odd steps from the second half, and the last 5 rows are looked up only
    at the final step, so rows sit out 1..steps-1 steps between lookups."""
    half = (rows - 5) // 2
    out = []
    for s in range(steps):
        lo, hi = (0, half) if s % 2 == 0 else (half, rows - 5)
        ids = rng.integers(lo, hi, B)
        if s == steps - 1:
            ids[:5] = np.arange(rows - 5, rows)
        out.append(ids)
    return out


SPECS = {
    "adagrad": (dict(kind="adagrad", eps=1e-10), "adagrad"),
    "rowwise_adagrad": (dict(kind="rowwise_adagrad", eps=1e-10), "rowwise"),
    "adam": (dict(kind="adam", eps=1e-8, betas=(0.9, 0.999), weight_decay=0.0, decoupled=False),
             "adam"),
    "adam_l2": (dict(kind="adam", eps=1e-8, betas=(0.8, 0.99), weight_decay=0.05,
                     decoupled=False), "adam"),
    "adamw_ref": (dict(kind="adam", eps=1e-6, betas=(0.9, 0.999), weight_decay=0.1,
                       decoupled=True), "adamw"),
    "adamw_nobc": (dict(kind="adam", eps=1e-6, betas=(0.9, 0.999), weight_decay=0.0,
                        decoupled=True, bias_correction=False), "adamw"),
}


def _oracle_step(kind, spec, P, G, S, t, lr):
    """Dense step of every table (all rows, like the reference's optimizer)."""
    for f in range(len(P)):
        p, g = P[f], G[f]
        if kind == "adagrad":
            ref.adagrad_step(p, g, S[f][0], lr, spec["eps"])
        elif kind == "rowwise":
            # the vector and the first-order column keep separate accumulators
            D = S[f][0].shape[1] if S[f][0].ndim == 2 else None
            pv, gv = p[:, :spec["D"]], g[:, :spec["D"]]
            ref.rowwise_adagrad_step(pv, gv, S[f][0], lr, spec["eps"])
            if p.shape[1] > spec["D"]:
                ref.adagrad_step(p[:, spec["D"]:], g[:, spec["D"]:], S[f][1], lr, spec["eps"])
        elif kind == "adam":
            ref.adam_step(p, g, S[f][0], S[f][1], t, lr, spec["betas"], spec["eps"],
                          spec["weight_decay"])
        else:
            ref.adamw_step(p, g, S[f][0], S[f][1], t, lr, spec["betas"], spec["eps"],
                           spec["weight_decay"], spec.get("bias_correction", True))


def _run(name, dtype, rows, B, steps, has_w, F, D=16, lr=0.05, seed=0, lr_sched=None):
    from pytorchrec_amd.embedding import gather
    spec, kind = SPECS[name]
    spec = dict(spec)
    rng = np.random.default_rng(seed)
    n = D + (1 if has_w else 0)
    init = [(rng.standard_normal((rows, n)) * 0.1).astype(np.float32) for _ in range(F)]
    if dtype == torch.bfloat16:
        init = [ref.bf16_bits_to_f32(ref.f32_to_bf16_bits(x)) for x in init]
    bank = _bank(rows, F, D, has_w, dtype, init)
    group = {"lr": lr}
    bank.use_fused_optimizer(spec.pop("kind"), group, **spec)
    bank.check_ids = False
    spec["D"] = D
    P = [x.astype(np.float64) for x in init]
    if kind == "rowwise":
        S = [(np.zeros(rows), np.zeros((rows, 1))) for _ in range(F)]
    else:
        S = [(np.zeros((rows, n)), np.zeros((rows, n))) for _ in range(F)]
    sched = [_ids_schedule(rng, rows, B, steps) for _ in range(F)]
    for s in range(steps):
        if lr_sched is not None:  # an LR scheduler changing the group's lr between steps
            lr = group["lr"] = lr_sched[s]
        ids = [torch.from_numpy(sched[f][s].astype(np.int32)).cuda() for f in range(F)]
        dy = (rng.standard_normal((B, F * D)) * 0.5).astype(np.float32)
        dyt = torch.from_numpy(dy).cuda()
        G = [np.zeros((rows, n)) for _ in range(F)]
        if has_w:
            dw = (rng.standard_normal(B) * 0.5).astype(np.float32)
            out, w_out = gather(bank, ids, out_dtype=torch.float32, with_w=True)
            loss = (out * dyt).sum() + (w_out[:, 0] * torch.from_numpy(dw).cuda()).sum()
            np.add.at(G[0][:, D], sched[0][s], dw.astype(np.float64))
        else:
            out = gather(bank, ids, out_dtype=torch.float32)
            loss = (out * dyt).sum()
        loss.backward()
        for f in range(F):
            np.add.at(G[f][:, :D], sched[f][s], dy[:, f * D:(f + 1) * D].astype(np.float64))
        _oracle_step(kind, spec, P, G, S, s + 1, lr)
    bank.flush_optimizer()
    torch.cuda.synchronize()
    return _table(bank, rows, F, D, has_w), P


@pytest.mark.parametrize("name", list(SPECS))
def test_fused_optimizer_fp32_matches_dense(gpu, name):
    got, want = _run(name, torch.float32, rows=61, B=96, steps=6, has_w=False, F=3)
    for f in range(3):
        np.testing.assert_allclose(got[f], want[f], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["adam", "adamw_ref", "adagrad"])
def test_fused_optimizer_lr_change_matches_dense(gpu, name):
    """The group's lr changes between steps (a scheduler): rows not looked up since
    the change took their missed zero-gradient Adam steps at the OLD lr in dense
    Adam, so the fused bank flushes them before installing the new lr."""
    got, want = _run(name, torch.float32, rows=61, B=96, steps=6, has_w=False, F=2, seed=9,
                     lr_sched=[0.05, 0.05, 0.02, 0.02, 0.1, 0.005])
    for f in range(2):
        np.testing.assert_allclose(got[f], want[f], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["adagrad", "rowwise_adagrad", "adam_l2", "adamw_ref"])
def test_fused_optimizer_first_order_column(gpu, name):
    """The first-order weight of a row (bank column D) gets its own state: an
    element of Adagrad / Adam, its own accumulator under row-wise Adagrad."""
    got, want = _run(name, torch.float32, rows=45, B=70, steps=5, has_w=True, F=1, seed=3)
    np.testing.assert_allclose(got[0], want[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["adagrad", "adamw_ref"])
def test_fused_optimizer_bf16_bank(gpu, name):
    """bf16 rows: fp32 optimizer math, one rounding of the row per update -- within
    a few bf16 ulps of the fp64 dense optimizer after 5 steps."""
    got, want = _run(name, torch.bfloat16, rows=61, B=96, steps=5, has_w=False, F=2, seed=5)
    for f in range(2):
        np.testing.assert_allclose(got[f], want[f], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("name", ["adagrad", "adam_l2"])
def test_fused_optimizer_large_batch_path(gpu, name):
    """More than MREC_BWD_MAX_BATCH lookups of a table (the large-batch path,
    emb_bwd_large.hip: hot rows summed in fixed point) with the fused optimizer."""
    got, want = _run(name, torch.float32, rows=3001, B=10000, steps=3, has_w=False, F=1,
                     seed=7, lr=0.01)
    np.testing.assert_allclose(got[0], want[0], rtol=1e-4, atol=1e-6)


def test_deepfm_adam_fused_equals_dense_grad(gpu):
    """IModel.compile with torch.optim.Adam fuses the table update; the same model
    stepping the table through a dense gradient and torch.optim.Adam ends with the
    same tables (after the fused optimizer's flush) and losses."""
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    F, R, B = 4, 53, 128
    sparse = [CategoricalColumnWithIdentity(R, f"c{f}") for f in range(F)]
    dense = [NumericColumn(f"d{j}") for j in range(3)]
    label = CategoricalColumnWithIdentity(2, "label")
    g = torch.Generator().manual_seed(0)
    batches = []
    for s in range(4):
        d = {c.feature_name: torch.randint(0, R // 2 if s % 2 == 0 else R, (B,), generator=g,
                                           dtype=torch.int32).cuda() for c in sparse}
        d.update({c.feature_name: torch.rand(B, generator=g).cuda() for c in dense})
        d["label"] = torch.randint(0, 2, (B,), generator=g).float().cuda()
        batches.append(d)
    tables, losses = [], []
    for fused in (True, False):
        m = DeepFM(sparse, dense, label, emb_size=16, layers=(32, 32), emb_dtype=torch.float32,
                   device=gpu, random_seed=11)
        m.compile(torch.optim.Adam(m.get_parameters(), lr=1e-2), BCEWithLogitsLoss(), [], gpu)
        assert m.embeddings.update == "adam"
        if not fused:
            m.embeddings.use_dense_grad()
        ls = [float(m.train_step(d)["loss"]) for d in batches]
        m.flush_embedding_optimizers()
        tables.append(m.embeddings.weight.detach().float().cpu().numpy())
        losses.append(ls)
    np.testing.assert_allclose(losses[0], losses[1], rtol=1e-5)
    np.testing.assert_allclose(tables[0], tables[1], rtol=1e-4, atol=1e-6)
