"""Row-sharded kernels on one GPU: W ranks simulated in one process (the
all-to-alls done by slicing), checked against the unsharded single-bank kernels
on the concatenated batch — bit-exact, since the owner's segment order (source
rank, then sample) is the concatenated batch's sample order.  Plus the autograd
path at W = 1 through a real ShardComm: a DeepFM train step identical to the
unsharded model's.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = [1000, 3, 70000, 257, 1, 4096]
D = 16


def _global_bank(gpu, dtype=torch.bfloat16):
    from pytorchrec_amd.embedding import EmbeddingBank, init_bank_
    bank = EmbeddingBank(ROWS, D, with_first_order=True, dtype=dtype, device=gpu)
    init_bank_(bank, std=0.5, generator=torch.Generator(device=gpu).manual_seed(1))
    bank.stochastic_rounding = False
    return bank


def _tables(bank):
    return [bank.weight[o:o + n] for o, n in zip(bank.row_offset, bank.category_nums)]


def _ids(gpu, B, seed, zipf=False):
    g = torch.Generator().manual_seed(seed)
    out = []
    for n in ROWS:
        if zipf:
            r = np.random.default_rng(seed + n)
            x = np.minimum(r.zipf(1.3, B) - 1, n - 1)
            out.append(torch.from_numpy(x.astype(np.int32)).to(gpu))
        else:
            out.append(torch.randint(0, n, (B,), generator=g, dtype=torch.int32).to(gpu))
    return out


def prefs_own(send, P, F, cap):
    """The sender's part prefixes of its table counts (int32 [P, F], exclusive)."""
    c = send.view(P, -1)[:, F * cap:F * cap + F].long()
    return (torch.cumsum(c, 1) - c).to(torch.int32)


def _exchange(sends, W):
    """all_to_all for W simulated ranks: out[r] = concat_s send[s] part r."""
    parts = [s.reshape(W, -1, *s.shape[1:]) if s.dim() > 1 else s.reshape(W, -1) for s in sends]
    return [torch.cat([p[r] for p in parts], 0).reshape(sends[r].shape) for r in range(W)]


@pytest.mark.parametrize("W,zipf,B,fused", [(2, False, 512, False), (4, False, 512, True),
                                            (4, True, 512, False), (3, True, 512, True),
                                            (2, False, 4096, True), (2, True, 4096, False),
                                            (8, False, 1024, True)])
def test_sharded_forward_backward_bit_exact(gpu, W, zipf, B, fused):
    """fused: the owner's plan runs inside the sender's interaction launch
    (owner_plan_job); else the standalone plan.  W * cap > 4096 entries takes the
    padded-view hash plan.  Skewed ids get cap = B (the default cap is sized for
    uniform ids)."""
    from pytorchrec_amd import embedding as E
    from pytorchrec_amd import sharding as S
    glob = _global_bank(gpu)
    banks = []
    for r in range(W):
        b = S.ShardedEmbeddingBank(ROWS, D, S.ShardComm(world=W, rank=r), with_first_order=True,
                                   dtype=torch.bfloat16, max_batch=B, device=gpu,
                                   cap=B if zipf else None)
        b.compact = False  # the slot exchange (its default cap counts lookups, not ids)
        b.load_global_(_tables(glob))
        b.stochastic_rounding = False
        banks.append(b)
    ids = [_ids(gpu, B, 10 + r, zipf) for r in range(W)]
    dense = [torch.rand(B, 13, device=gpu) for _ in range(W)]
    dense_w = torch.randn(13, device=gpu)
    bias = torch.randn(1, device=gpu)
    x0_cols = 104 + 16  # 6*16 + 13 -> 109 -> 112; use a wider pad
    # ---- forward
    sends, poss = zip(*[S.shard_bucketize(banks[r], ids[r]) for r in range(W)])
    for r in range(W):
        ref_send, ref_pos = S.cpu_bucketize(banks[r], [t.cpu() for t in ids[r]])
        assert torch.equal(sends[r].cpu(), ref_send) and torch.equal(poss[r].cpu(), ref_pos)
    recvs = _exchange(list(sends), W)
    rows = _exchange([S.shard_gather(banks[r], recvs[r]) for r in range(W)], W)
    plans, outs = [], []
    for r in range(W):
        job, plan, keep = (S.owner_plan_job(banks[r], recvs[r]) if fused else (None, None, None))
        outs.append(S.shard_interact(banks[r], rows[r], poss[r], dense[r], dense_w, bias, True,
                                     True, x0_cols, torch.bfloat16, plan_job=job))
        plans.append(plan if fused else S.owner_plan(banks[r], recvs[r]))
        del keep
    for r in range(W):
        banks[r].check_flags()
    with torch.no_grad():
        for r in range(W):
            x0, logit = E.interact(glob, ids[r], dense[r], dense_w, bias, True, True, x0_cols,
                                   torch.bfloat16)
            assert torch.equal(outs[r][0], x0)
            assert torch.equal(outs[r][1], logit)
    # ---- backward: given dx0 / dlogit per rank, SGD lr on the owners
    lr = 0.5
    dx0 = [torch.randn(B, x0_cols, device=gpu).to(torch.bfloat16) for _ in range(W)]
    dl = [torch.randn(B, device=gpu) for _ in range(W)]
    gs = [S.shard_lookup_grad(banks[r], poss[r], B, dx=dx0[r], dfm=dl[r], fm_sum=outs[r][2],
                              x0=outs[r][0], dw=dl[r]) for r in range(W)]
    grecv = _exchange(gs, W)
    for r in range(W):
        S.owner_apply(banks[r], plans[r], grecv[r], lr)
        banks[r].check_flags()
    # reference: one bank, concatenated batch (rank 0's samples first)
    glob.use_fused_sgd(lr)
    cat = lambda xs: torch.cat(xs, 0)
    ids_all = [cat([ids[r][f] for r in range(W)]) for f in range(len(ROWS))]
    fm_all = cat([o[2] for o in outs])
    x0_all = cat([o[0] for o in outs])
    E._backward_into_bank(glob, ids_all, W * B, None, dx=cat(dx0), dfm=cat(dl), fm_sum=fm_all,
                          x0=x0_all, dw=cat(dl))
    cols = D + 1
    for r in range(W):
        for f, (o, n) in enumerate(zip(banks[r].row_offset, banks[r].category_nums)):
            want = glob.weight[glob.row_offset[f]:glob.row_offset[f] + ROWS[f]][r::W, :cols]
            got = banks[r].weight[o:o + n, :cols]
            assert torch.equal(got, want), (r, f)


def test_sharded_overflow_is_raised(gpu):
    from pytorchrec_amd import sharding as S
    bank = S.ShardedEmbeddingBank([100], D, S.ShardComm(world=2, rank=0), dtype=torch.bfloat16,
                                  cap=4, device=gpu)
    ids = [torch.zeros(9, dtype=torch.int32, device=gpu)]  # 9 ids for owner 0, cap 4
    S.shard_bucketize(bank, ids)
    with pytest.raises(RuntimeError, match="overflow"):
        bank.check_flags()
    S.shard_bucketize(bank, [torch.tensor([100], dtype=torch.int32, device=gpu)])
    with pytest.raises(IndexError):
        bank.check_flags()


def _deepfm(gpu, sharded, emb_dtype=torch.bfloat16, max_batch=256):
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    from pytorchrec_amd.sharding import ShardComm, sharded_tables
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{i}") for i, n in enumerate(ROWS)]
    dense = [NumericColumn(f"c_n_I{i}") for i in range(13)]
    label = CategoricalColumnWithIdentity(2, "label")
    torch.manual_seed(3)
    if sharded:
        with sharded_tables(ShardComm(world=1, rank=0), max_batch=max_batch):
            m = DeepFM(sparse, dense, label, emb_size=D, layers=(64, 32), emb_dtype=emb_dtype,
                       random_seed=5, device=gpu)
    else:
        m = DeepFM(sparse, dense, label, emb_size=D, layers=(64, 32), emb_dtype=emb_dtype,
                   random_seed=5, device=gpu)
    return m


def test_world1_sharded_deepfm_step_equals_unsharded(gpu):
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    a, b = _deepfm(gpu, False), _deepfm(gpu, True)
    b.load_state_dict(a.state_dict())
    data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, 256, 3))}
    g = torch.Generator().manual_seed(4)
    for i in range(13):
        data[f"c_n_I{i}"] = torch.rand(256, generator=g).to(gpu)
    data["label"] = (torch.rand(256, generator=g) < 0.25).to(torch.int32).to(gpu)
    for m in (a, b):
        opt = torch.optim.SGD(m.get_parameters(), lr=0.05)
        m.compile(opt, BCEWithLogitsLoss(), [], gpu)
    la = [float(a.train_step(data)["loss"].detach()) for _ in range(2)]
    lb = [float(b.train_step(data)["loss"].detach()) for _ in range(2)]
    assert la == lb
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k


def test_world1_sharded_large_batch_default_cap_equals_unsharded(gpu):
    """a world-1 sharded bank built for B = 16,384 takes the slot exchange
    with a defaulted cap sized for the WHOLE batch (the slot bucketize does not
    chunk), so nothing overflows and the owner's view (W * cap > 8,192 entries)
    takes the large-batch owner apply: two steps bit-identical to the unsharded
    model."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    B = 16384
    a, b = _deepfm(gpu, False), _deepfm(gpu, True, max_batch=B)
    assert b.embeddings.cap >= B and not b.embeddings.use_compact(B)
    b.load_state_dict(a.state_dict())
    data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, B, 5))}
    g = torch.Generator().manual_seed(6)
    for i in range(13):
        data[f"c_n_I{i}"] = torch.rand(B, generator=g).to(gpu)
    data["label"] = (torch.rand(B, generator=g) < 0.25).to(torch.int32).to(gpu)
    for m in (a, b):
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
    la = [float(a.train_step(data)["loss"].detach()) for _ in range(2)]
    lb = [float(b.train_step(data)["loss"].detach()) for _ in range(2)]
    b.embeddings.check_flags()
    assert la == lb
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k


@pytest.mark.parametrize("opt", ["adagrad", "rowwise_adagrad", "adam", "adamw"])
def test_world1_sharded_fused_optimizers_equal_unsharded(gpu, opt):
    """Row-sharded tables train with the fused optimizers too (owner apply with the
    gradient scale 1/W): at W = 1 the sharded model equals the unsharded one over
    batches that leave rows out for a step (the lazy Adam's catch-up on reads and
    updates on both paths)."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.optim import AdamW, RowWiseAdagrad
    a, b = _deepfm(gpu, False), _deepfm(gpu, True)
    b.load_state_dict(a.state_dict())
    batches = []
    for s in range(3):
        data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, 256, 20 + s))}
        g = torch.Generator().manual_seed(30 + s)
        for i in range(13):
            data[f"c_n_I{i}"] = torch.rand(256, generator=g).to(gpu)
        data["label"] = (torch.rand(256, generator=g) < 0.25).to(torch.int32).to(gpu)
        batches.append(data)
    make = {"adagrad": lambda p: torch.optim.Adagrad(p, lr=0.05),
            "rowwise_adagrad": lambda p: RowWiseAdagrad(p, lr=0.05),
            "adam": lambda p: torch.optim.Adam(p, lr=0.01, weight_decay=0.01),
            "adamw": lambda p: AdamW(p, lr=0.01, weight_decay=0.01)}[opt]
    for m in (a, b):
        m.compile(make(m.get_parameters()), BCEWithLogitsLoss(), [], gpu)
    kind = "adam" if opt == "adamw" else opt
    assert a.embeddings.update == kind and b.embeddings.update == kind
    la = [float(a.train_step(d)["loss"].detach()) for d in batches]
    lb = [float(b.train_step(d)["loss"].detach()) for d in batches]
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        torch.testing.assert_close(sa[k].float(), sb[k].float(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("opt", ["adam", "adamw"])
def test_world1_compact_exchange_lazy_adam_equals_unsharded(gpu, opt):
    """A fused lazy Adam bank on the COMPACT exchange (ABI 25: the owner's wire
    gather catches every row up to the current step as it packs the record; the
    owner's apply reads the gradient records in place and steps Adam): at W = 1
    with fp32 tables (fp32 records: the wire is exact) the sharded model equals the
    unsharded one over batches that leave rows out for a step, i.e. the forward
    reads the caught-up rows and the updates replay the missed steps the same way."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.optim import AdamW
    a, b = _deepfm(gpu, False, torch.float32), _deepfm(gpu, True, torch.float32)
    b.load_state_dict(a.state_dict())
    b.embeddings.compact = "always"
    batches = []
    for s in range(4):
        data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, 256, 60 + s))}
        g = torch.Generator().manual_seed(70 + s)
        for i in range(13):
            data[f"c_n_I{i}"] = torch.rand(256, generator=g).to(gpu)
        data["label"] = (torch.rand(256, generator=g) < 0.25).to(torch.int32).to(gpu)
        batches.append(data)
    make = {"adam": lambda p: torch.optim.Adam(p, lr=0.01, weight_decay=0.01),
            "adamw": lambda p: AdamW(p, lr=0.01, weight_decay=0.01)}[opt]
    for m in (a, b):
        m.compile(make(m.get_parameters()), BCEWithLogitsLoss(), [], gpu)
    assert a.embeddings.update == "adam" and b.embeddings.update == "adam"
    assert b.embeddings.use_compact(256)
    la = [float(a.train_step(d)["loss"].detach()) for d in batches]
    lb = [float(b.train_step(d)["loss"].detach()) for d in batches]
    b.embeddings.check_flags()
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        torch.testing.assert_close(sa[k].float(), sb[k].float(), rtol=1e-5, atol=1e-6)


@pytest.fixture
def rccl_world1(gpu):
    """A real one-rank RCCL process group (collectives forced at world 1)."""
    import os
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = os.environ.get("MREC_TEST_PORT", "29613")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    try:
        yield
    finally:
        dist.destroy_process_group()


def test_world1_rccl_dp_sharded_deepfm_step_equals_unsharded(gpu, rccl_world1):
    """Row-sharded tables + data-parallel dense tower with every collective issued
    (all_to_all x3, one flat all_reduce + mrec_sgd_multi) == the single-process
    fused step, bit for bit (the sum over one rank is exact)."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.sharding import ShardComm
    a, b = _deepfm(gpu, False), _deepfm(gpu, True)
    b.load_state_dict(a.state_dict())
    b.embeddings.comm = ShardComm(force_collectives=True)
    b.distribute(ShardComm(force_collectives=True))
    data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, 256, 7))}
    g = torch.Generator().manual_seed(8)
    for i in range(13):
        data[f"c_n_I{i}"] = torch.rand(256, generator=g).to(gpu)
    data["label"] = (torch.rand(256, generator=g) < 0.25).to(torch.int32).to(gpu)
    for m in (a, b):
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
    assert b._dp_flat is not None and len(b._dp_flat[1]) == 8  # 2 MLP + head (W, b), w_dense, bias
    la = [float(a.train_step(data)["loss"].detach()) for _ in range(3)]
    lb = [float(b.train_step(data)["loss"].detach()) for _ in range(3)]
    assert la == lb
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k


def _batches(gpu, n, B=256, seed=90):
    out = []
    for s in range(n):
        data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, B, seed + s))}
        g = torch.Generator().manual_seed(seed + 50 + s)
        for i in range(13):
            data[f"c_n_I{i}"] = torch.rand(B, generator=g).to(gpu)
        data["label"] = (torch.rand(B, generator=g) < 0.25).to(torch.int32).to(gpu)
        out.append(data)
    return out


def test_world1_rccl_compact_inline_dense_sgd_bit_identical(gpu, rccl_world1):
    """ABI 28: a data-parallel dense tower over the compact exchange all-reduces its
    flat gradient right before the owner apply, and the dense SGD tiles ride in that
    launch (IModel._dp_inline_sgd -> mrec_emb_bwd_apply_wire_sgd).  Against the
    separate mrec_sgd_multi launch after the backward (the hook removed): the same
    losses and parameters bit for bit over three steps, every collective issued."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.sharding import ShardComm
    a, b = _deepfm(gpu, True), _deepfm(gpu, True)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        m.embeddings.compact = "always"
        m.embeddings.comm = ShardComm(force_collectives=True)
        m.distribute(ShardComm(force_collectives=True))
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
    assert getattr(b.embeddings, "dp_inline_sgd", None) is not None
    del a.embeddings.dp_inline_sgd  # a: the flat step's own mrec_sgd_multi launch
    batches = _batches(gpu, 3)
    la = [float(a.train_step(d)["loss"].detach()) for d in batches]
    lb = [float(b.train_step(d)["loss"].detach()) for d in batches]
    assert b._dp_sgd_table is not None and a._dp_sgd_table is None  # b went inline
    assert la == lb
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k


def test_world1_mrec_comm_sharded_step_equals_unsharded(gpu):
    """The C-ABI communicator (mrec_comm_init / mrec_a2a_* / mrec_allreduce_sum_f32,
    RCCL opened by libmrec, no torch.distributed at all) drives the row-sharded +
    data-parallel step at world 1 with every exchange issued: bit-identical to the
    single-process step; the step captured in a HIP graph replays, and once the
    graph is released mrec_comm_destroy returns."""
    import gc
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.sharding import MrecComm
    comm = MrecComm(world=1, rank=0)
    a, b = _deepfm(gpu, False), _deepfm(gpu, True)
    b.load_state_dict(a.state_dict())
    b.embeddings.comm = comm
    b.distribute(comm)
    data = {f"c_c_C{i}": t for i, t in enumerate(_ids(gpu, 256, 9))}
    g = torch.Generator().manual_seed(10)
    for i in range(13):
        data[f"c_n_I{i}"] = torch.rand(256, generator=g).to(gpu)
    data["label"] = (torch.rand(256, generator=g) < 0.25).to(torch.int32).to(gpu)
    for m in (a, b):
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
        for bank in m.embedding_banks():
            # RNE updates: a replayed graph reuses its captured host seed, an eager step
            # draws a new one, so stochastic rounding would differ between the two
            bank.stochastic_rounding = False
    la = [float(a.train_step(data)["loss"].detach()) for _ in range(3)]
    lb = [float(b.train_step(data)["loss"].detach()) for _ in range(3)]
    assert la == lb
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k
    for bank in b.embedding_banks():
        bank.check_ids = False
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.train_step(data)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        b.train_step(data)
    for _ in range(2):
        graph.replay()
    a.train_step(data)
    a.train_step(data)
    a.train_step(data)
    torch.cuda.synchronize()
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k
    del graph
    gc.collect()
    torch.cuda.synchronize()
    comm.close()


def test_sgd_multi_matches_torch_and_weight_prep(gpu):
    """mrec_sgd_multi: w -= lr g for several shapes in one launch, images equal
    to mrec_weight_prep of the updated weight (pad columns zero)."""
    from pytorchrec_amd import _mrec
    from pytorchrec_amd.dense import weight_prep
    shapes = [(400, 429), (1, 400), (13,), (1,), (37, 5)]
    ws, jobs, keep = [], [], []
    for sh in shapes:
        w = torch.randn(*sh, device=gpu)
        n, k = (1, w.numel()) if w.dim() < 2 else w.shape
        ld = (k + 7) // 8 * 8
        gbuf = torch.randn(n, ld, device=gpu)
        want = (w.reshape(n, k).double() - 0.25 * gbuf[:, :k].double()).float()
        img = None
        if w.dim() == 2:
            img = (torch.full((n, (k + 7) // 8 * 8), 7, dtype=torch.bfloat16, device=gpu),
                   torch.full((k, (n + 7) // 8 * 8), 7, dtype=torch.bfloat16, device=gpu))
        jobs.append(_mrec.SgdJob(w.data_ptr(), gbuf.data_ptr(), n, k, k, ld, 0.25,
                                 _mrec.ptr(img[0]) if img else None, img[0].stride(0) if img else 0,
                                 _mrec.ptr(img[1]) if img else None, img[1].stride(0) if img else 0))
        ws.append((w, img, want))
        keep.append(gbuf)
    arr = (_mrec.SgdJob * len(jobs))(*jobs)
    _mrec.call("mrec_sgd_multi", len(jobs), arr, _mrec.stream_handle())
    for w, img, want in ws:
        n, k = want.shape
        torch.testing.assert_close(w.reshape(n, k), want, rtol=0, atol=1e-6)
        if img is not None:
            wr, wt = weight_prep(w)
            assert torch.equal(img[0], wr) and torch.equal(img[1], wt)


# ---------------------------------------------------------------------------
# compact exchange (ABI 19): distinct ids, 36-B records, summed gradients
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("W,zipf,B,big", [(2, False, 512, False), (4, True, 512, False),
                                          (8, False, 1024, False), (3, True, 4096, False),
                                          (8, True, 4096, False), (2, False, 8192, False),
                                          (8, True, 4096, True), (4, False, 8192, True),
                                          (8, True, 16384, True)])
def test_compact_exchange_simulated_bit_exact(gpu, W, zipf, B, big):
    """W ranks simulated in one process (all-to-alls by slicing), every stage checked:
      * bucketize_dedup == its CPU restatement (cpu_bucketize_dedup): the distinct
        ids per (owner, table) in first-lookup order, every lookup's slot, counts;
      * the records unpacked at the sender hold exactly the looked-up rows (bit
        copy) and the interaction over them == the unsharded bank's (bit-exact);
      * the sender's per-slot gradient sums == rank r's own dense gradient of the
        unsharded bank (same kernels: fixed ascending order, rounded once to the
        table dtype -- the wire format);
      * the owner's sum over the senders (DENSE_GRAD) == the fp32 sum of the ranks'
        bf16 gradients in rank order, rounded once (bit-exact);
      * with fused SGD the owners' rows are within 1 bf16 ulp of that sum applied.
    ``big``: cap = B, so the owner's exchange view (W * cap entries per table, up to
    32,768) exceeds one plan workgroup and the owner takes the large-batch bucketed
    path over the received records / fp32 slots (owner_apply_large, ABI 25): the
    same sums (a row has <= W entries, summed in sender order), bit-exact.
    B = 16,384 per rank (Zipf, W = 8): each rank's batch goes out as 2 chunks of
    8,192 (sub-senders: every message has W x 2 parts, mrec_shard_bucketize_dedup_ex);
    each chunk's slot sums == the dense gradient of that chunk alone, and the owner's
    sum runs over (rank, chunk) in that order.
    Per-rank bytes on the wire are checked against the slot exchange."""
    from pytorchrec_amd import _mrec
    from pytorchrec_amd import embedding as E
    from pytorchrec_amd import sharding as S
    glob = _global_bank(gpu)
    banks = []
    for r in range(W):
        b = S.ShardedEmbeddingBank(ROWS, D, S.ShardComm(world=W, rank=r), with_first_order=True,
                                   dtype=torch.bfloat16, max_batch=B, device=gpu,
                                   cap=min(B, 8192) if big else (min(B, 8192 // W) if zipf else None))
        b.load_global_(_tables(glob))
        b.stochastic_rounding = False
        assert b.use_compact(B)
        banks.append(b)
    ids = [_ids(gpu, B, 40 + r, zipf) for r in range(W)]
    dense = [torch.rand(B, 13, device=gpu) for _ in range(W)]
    dense_w = torch.randn(13, device=gpu)
    bias = torch.randn(1, device=gpu)
    x0_cols = 112
    F = len(ROWS)
    sends, poss = zip(*[S.shard_bucketize_dedup(banks[r], ids[r]) for r in range(W)])
    for r in range(W):
        ref_send, ref_pos = S.cpu_bucketize_dedup(banks[r], [t.cpu() for t in ids[r]])
        assert torch.equal(sends[r].cpu(), ref_send) and torch.equal(poss[r].cpu(), ref_pos), r
    recvs = _exchange(list(sends), W)
    P = banks[0].parts(B)  # W x chunks
    CB = banks[0].chunk_batch
    chunks = [(s0, min(CB, B - s0)) for s0 in range(0, B, CB)]
    assert P == W * len(chunks)
    prefs = [torch.empty(P, len(ROWS), dtype=torch.int32, device=gpu) for _ in range(W)]
    wires = _exchange([S.shard_gather_wire(banks[r], recvs[r], pref=prefs[r], parts=P)
                       for r in range(W)], W)
    n = P * F * banks[0].cap
    rows, gsums, outs, plans, oplans, sprefs = [], [], [], [], [], []
    for r in range(W):
        rr = torch.empty(n, banks[r].row_stride, dtype=torch.bfloat16, device=gpu)
        gs = torch.empty_like(rr)
        sprefs.append(torch.empty(P, F, dtype=torch.int32, device=gpu))
        S.shard_wire_unpack(banks[r], wires[r], sends[r], rr, zero=gs, parts=P, pref=sprefs[r])
        rows.append(rr)
        gsums.append(gs)
        fuse = B <= 4096
        job, sp, keep = S.sender_plan_job(banks[r], rr, poss[r]) if fuse else (None, None, None)
        outs.append(S.shard_interact(banks[r], rr, poss[r], dense[r], dense_w, bias, True, True,
                                     x0_cols, torch.bfloat16, plan_job=job))
        del keep
        if fuse and S.records_direct(banks[r]):
            # ABI 28: the interaction over the received records itself (no unpack) --
            # same outputs, the same slot rows left behind, the same part prefixes
            rr2 = torch.empty_like(rr)
            sp2 = torch.full((P, F), -7, dtype=torch.int32, device=gpu)
            rec = _mrec.WireRows(wires[r].data_ptr(), banks[r].wire_bytes(), sends[r].data_ptr(), P,
                                 banks[r].cap, banks[r].cap_rows, sp2.data_ptr(),
                                 banks[r].flags().data_ptr())
            job2, _, keep2 = S.sender_plan_job(banks[r], rr2, poss[r])
            out2 = S.shard_interact(banks[r], rr2, poss[r], dense[r], dense_w, bias, True, True,
                                    x0_cols, torch.bfloat16, plan_job=job2, rec=rec)
            del keep2
            for a_, b_ in zip(out2, outs[-1]):
                assert torch.equal(a_, b_), r
            looked = poss[r].reshape(-1).long()
            looked = looked[looked >= 0]
            assert torch.equal(rr2[looked].view(torch.int16), rr[looked].view(torch.int16)), r
            assert torch.equal(sp2, sprefs[r]), r
        plans.append([(0, B, sp)] if fuse else S.sender_plans(banks[r], rr, poss[r]))
        large = not S.owner_view_fits_hash(banks[r], P)  # W * cap entries past one plan
        assert large or not big
        oplans.append(None if large else S.owner_plan(banks[r], recvs[r], banks[r].part, P))
    for r in range(W):
        banks[r].check_flags()
        gw = glob.weight
        for f in range(F):
            p = poss[r][f].long()
            want = gw[glob.row_offset[f] + ids[r][f].long(), :D + 1]
            assert torch.equal(rows[r][p, :D + 1], want), (r, f)
        with torch.no_grad():
            x0, logit = E.interact(glob, ids[r], dense[r], dense_w, bias, True, True, x0_cols,
                                   torch.bfloat16)
        assert torch.equal(outs[r][0], x0) and torch.equal(outs[r][1], logit), r
    # ---- backward
    dx0 = [torch.randn(B, x0_cols, device=gpu).to(torch.bfloat16) for _ in range(W)]
    dl = [torch.randn(B, device=gpu) for _ in range(W)]
    rank_grads = []  # (rank, chunk) order = the owners' summation order
    for r in range(W):
        for s0, nc in chunks:
            sl = (lambda t: t[s0:s0 + nc])  # noqa: E731
            sp = [p_ for p_ in plans[r] if p_[0] == s0][0][2]
            S.sender_grad_sums(banks[r], rows[r], poss[r][:, s0:s0 + nc], sp, gsums[r],
                               dx=sl(dx0[r]), dfm=sl(dl[r]), fm_sum=sl(outs[r][2]),
                               x0=sl(outs[r][0]), dw=sl(dl[r]))
            # reference: the chunk's dense gradient of the unsharded bank (bf16, same kernels)
            ref = E.EmbeddingBank(ROWS, D, with_first_order=True, dtype=torch.bfloat16,
                                  update="dense", device=gpu)
            with torch.no_grad():
                ref.weight.copy_(glob.weight)
            ids_c = [sl(t) for t in ids[r]]
            gref = E._backward_into_bank(ref, ids_c, nc, None, dx=sl(dx0[r]), dfm=sl(dl[r]),
                                         fm_sum=sl(outs[r][2]), x0=sl(outs[r][0]), dw=sl(dl[r]))
            rank_grads.append(gref)
            for f in range(F):
                p = poss[r][f, s0:s0 + nc].long()
                want = gref[glob.row_offset[f] + ids_c[f].long(), :D + 1]
                assert torch.equal(gsums[r][p, :D + 1], want), (r, s0, f)
    packed = [S.shard_wire_pack(banks[r], gsums[r], sends[r], parts=P) for r in range(W)]
    if B <= 4096:  # one hash-layout chunk: the sums written straight as records (ABI 26)
        rb = banks[0].wire_bytes()
        for r in range(W):
            recs = S.sender_grad_records(banks[r], rows[r], poss[r], plans[r][0][2], sprefs[r],
                                         parts=P, dx=dx0[r], dfm=dl[r], fm_sum=outs[r][2],
                                         x0=outs[r][0], dw=dl[r])
            cnt = sends[r].view(P, -1)[:, F * banks[r].cap:].sum(1).clamp(max=banks[r].cap_rows)
            for p_ in range(P):
                k = int(cnt[p_]) * rb
                assert torch.equal(recs[p_, :k], packed[r][p_, :k]), (r, p_)
            assert torch.equal(sprefs[r], prefs_own(sends[r], P, F, banks[r].cap)), r
    wire_g = _exchange(packed, W)
    tot = torch.zeros_like(rank_grads[0], dtype=torch.float32)
    for g in rank_grads:  # the owners' order: source rank 0, 1, ...
        tot += g.float()
    for r in range(W):
        g_recv = torch.empty(n, banks[r].g_ld, dtype=torch.float32, device=gpu)
        S.shard_wire_unpack(banks[r], wire_g[r], recvs[r], g_recv, to_f32=True, parts=P)
        own = torch.zeros_like(banks[r].weight)
        own_w = torch.zeros_like(banks[r].weight)
        if oplans[r] is None:  # the large-batch path over the slots, then the records in place
            S.owner_apply_large(banks[r], recvs[r], banks[r].part, g_occ=g_recv, grad=own,
                                parts=P)
            S.owner_apply_large(banks[r], recvs[r], banks[r].part, wire_g=wire_g[r],
                                pref=prefs[r], grad=own_w, parts=P)
        else:
            S.owner_apply(banks[r], oplans[r], g_recv, grad=own)
            # the same sums read from the received records in place (no unpack)
            S.owner_apply_wire(banks[r], oplans[r], wire_g[r], prefs[r], grad=own_w, parts=P)
        banks[r].check_flags()
        assert torch.equal(own_w.view(torch.int16), own.view(torch.int16)), r
        for f, (o, cnt) in enumerate(zip(banks[r].row_offset, banks[r].category_nums)):
            want = tot[glob.row_offset[f]:glob.row_offset[f] + ROWS[f]][r::W, :D + 1]
            assert torch.equal(own[o:o + cnt, :D + 1], want.to(torch.bfloat16)), (r, f)
        # fused SGD from the same sums: within one bf16 ulp of w - lr * sum
        lr = 0.5
        before = banks[r].weight.detach().clone()
        if oplans[r] is None:
            S.owner_apply_large(banks[r], recvs[r], banks[r].part, wire_g=wire_g[r],
                                pref=prefs[r], lr=lr, parts=P)
        else:
            S.owner_apply_wire(banks[r], oplans[r], wire_g[r], prefs[r], lr, parts=P)
        after_wire = banks[r].weight.detach().clone()
        with torch.no_grad():
            banks[r].weight.copy_(before)
        if oplans[r] is None:
            S.owner_apply_large(banks[r], recvs[r], banks[r].part, g_occ=g_recv, lr=lr, parts=P)
        else:
            S.owner_apply(banks[r], oplans[r], g_recv, lr)
        banks[r].check_flags()
        # bitwise, pad columns included (zeroed at allocation)
        assert torch.equal(banks[r].weight.view(torch.int16), after_wire.view(torch.int16)), r
        for f, (o, cnt) in enumerate(zip(banks[r].row_offset, banks[r].category_nums)):
            g = tot[glob.row_offset[f]:glob.row_offset[f] + ROWS[f]][r::W, :D + 1].double()
            w0 = before[o:o + cnt, :D + 1].double()
            want = w0 - lr * g
            got = banks[r].weight[o:o + cnt, :D + 1].double()
            ulp = torch.from_numpy(np.spacing(np.abs(want.cpu().numpy()).astype(np.float32))
                                   .astype(np.float64)).to(gpu) * 2 ** 16  # bf16 ulp
            assert bool(((got - want).abs() <= ulp * 1.0001 + 1e-30).all()), (r, f)
    # bytes on the wire per rank and direction vs the slot exchange
    rb = banks[0].wire_bytes()
    compact = W * banks[0].cap_rows * rb
    slot = W * F * banks[0].cap * banks[0].row_stride * 2
    assert compact < slot



def test_c5_sized_tables_compact_exchange_w8(gpu):
    """C5's 100,000,000-row tables on the row-sharded path: W = 8
    ranks simulated in one process, 2 tables x 1e8 rows (each rank's shard 12.5 M
    rows per table, byte offsets past 2^31), B = 4096 uniform ids per rank over the
    whole range plus the last rows.  Compact exchange: every record the sender
    unpacks is bit-exactly the owner's row; the senders' per-slot gradient sums
    (dx only) equal the fp32 sum of the rank's lookups in ascending sample order,
    rounded once to bf16; the owners' fused SGD moves each touched row to
    w - lr * (rank-order fp32 sum of those) within one bf16 ulp."""
    from pytorchrec_amd import sharding as S
    W, B, R, F = 8, 4096, 100_000_000, 2
    rows_g = [R, R]
    banks = []
    for r in range(W):
        b = S.ShardedEmbeddingBank(rows_g, D, S.ShardComm(world=W, rank=r), with_first_order=True,
                                   dtype=torch.bfloat16, max_batch=B, device=gpu)
        with torch.no_grad():
            b.weight.copy_(torch.randn(b.weight.shape, device=gpu,
                                       generator=torch.Generator(device=gpu).manual_seed(r)))
        b.stochastic_rounding = False
        assert b.use_compact(B)
        banks.append(b)
    g = torch.Generator().manual_seed(5)
    ids = []
    for r in range(W):
        t = [torch.randint(0, R, (B,), generator=g, dtype=torch.int32) for _ in range(F)]
        t[0][:W] = torch.arange(R - W, R, dtype=torch.int32)  # the last row of every shard
        ids.append([x.to(gpu) for x in t])
    sends, poss = zip(*[S.shard_bucketize_dedup(banks[r], ids[r]) for r in range(W)])
    recvs = _exchange(list(sends), W)
    ojobs = [S.owner_plan_job(banks[r], recvs[r], banks[r].part) for r in range(W)]
    wires = _exchange([S.shard_gather_wire(banks[r], recvs[r], plan_job=ojobs[r][0])
                       for r in range(W)], W)
    n = W * F * banks[0].cap
    rows, gsums = [], []
    for r in range(W):
        rr = torch.empty(n, banks[r].row_stride, dtype=torch.bfloat16, device=gpu)
        gs = torch.empty_like(rr)
        S.shard_wire_unpack(banks[r], wires[r], sends[r], rr, zero=gs)
        rows.append(rr)
        gsums.append(gs)
        banks[r].check_flags()
        for f in range(F):
            idl = ids[r][f].long()
            own, loc = idl % W, idl // W
            want = torch.empty(B, D + 1, dtype=torch.bfloat16, device=gpu)
            for o in range(W):
                m = own == o
                want[m] = banks[o].weight[banks[o].row_offset[f] + loc[m], :D + 1]
            assert torch.equal(rows[r][poss[r][f].long(), :D + 1], want), (r, f)
    # backward: dx only (gradient of lookup (b, f) = dx0[b, 16 f .. 16 f + 16], w: 0)
    x0_cols = F * D
    dx0 = [torch.randn(B, x0_cols, device=gpu).to(torch.bfloat16) for _ in range(W)]
    tot = {}  # global (f, id) -> fp32 rank-order sum of the ranks' bf16 sums
    for r in range(W):
        plan = S.sender_plan(banks[r], rows[r], poss[r])
        S.sender_grad_sums(banks[r], rows[r], poss[r], plan, gsums[r], dx=dx0[r])
        dxr = dx0[r].float().cpu().numpy()
        for f in range(F):
            idr = ids[r][f].cpu().numpy()
            order = np.argsort(idr, kind="stable")
            uniq, start = np.unique(idr[order], return_index=True)
            ends = np.append(start[1:], len(order))
            pos_r = poss[r][f].cpu().numpy()
            got = gsums[r][torch.from_numpy(pos_r[order[start]]).long().to(gpu), :D].float().cpu().numpy()
            for k, (s0, s1) in enumerate(zip(start, ends)):
                acc = np.zeros(D, np.float32)
                for b in order[s0:s1]:  # ascending sample order
                    acc += dxr[b, f * D:(f + 1) * D]
                want = torch.from_numpy(acc).to(torch.bfloat16).float().numpy()
                assert np.array_equal(got[k], want), (r, f, uniq[k])
                key = (f, int(uniq[k]))
                tot[key] = tot.get(key, np.zeros(D, np.float32)) + want
    wire_g = _exchange([S.shard_wire_pack(banks[r], gsums[r], sends[r]) for r in range(W)], W)
    lr = 0.5
    for r in range(W):
        g_recv = torch.empty(n, banks[r].g_ld, dtype=torch.float32, device=gpu)
        S.shard_wire_unpack(banks[r], wire_g[r], recvs[r], g_recv, to_f32=True)
        before = banks[r].weight.detach().clone()
        S.owner_apply(banks[r], ojobs[r][1], g_recv, lr)
        banks[r].check_flags()
        keys = [k for k in tot if k[1] % W == r]
        idx = torch.tensor([banks[r].row_offset[f] + i // W for f, i in keys], device=gpu)
        w0 = before[idx, :D].double()
        want = w0 - lr * torch.from_numpy(np.stack([tot[k] for k in keys])).double().to(gpu)
        got = banks[r].weight[idx, :D].double()
        ulp = torch.from_numpy(np.spacing(np.abs(want.cpu().numpy()).astype(np.float32))
                               .astype(np.float64)).to(gpu) * 2 ** 16
        assert bool(((got - want).abs() <= ulp * 1.0001 + 1e-30).all()), r
        # rows nobody looked up (a sample of them) keep their bits
        probe = torch.randint(0, banks[r].weight.shape[0], (4096,), device=gpu)
        touched = torch.zeros(banks[r].weight.shape[0], dtype=torch.bool, device=gpu)
        touched[idx] = True
        keep = probe[~touched[probe]]
        assert torch.equal(banks[r].weight[keep], before[keep]), r
        del before
    del banks, rows, gsums
    torch.cuda.empty_cache()


def test_compact_cap_rows_overflow_raised_and_clipped_rows_untouched(gpu):
    """a part whose distinct ids exceed cap_rows has its records clipped;
    the overflow is raised (its own message), and the owner's apply reading the
    gradient records in place gives the clipped entries a zero gradient -- their rows
    stay unchanged, never another entry's record (emb_apply.h wire_grad)."""
    from pytorchrec_amd import sharding as S
    n_rows, B = 1000, 64
    bank = S.ShardedEmbeddingBank([n_rows], D, S.ShardComm(world=1, rank=0), dtype=torch.float32,
                                  max_batch=B, cap=B, device=gpu)
    with torch.no_grad():
        bank.weight.copy_(torch.randn_like(bank.weight))
    bank.cap_rows = 8  # 40 distinct ids below: entries 8.. are clipped
    ids = [torch.arange(40, dtype=torch.int32, device=gpu).repeat(2)[:B] * 7]
    send, pos = S.shard_bucketize_dedup(bank, ids)
    recv = send  # world 1
    pref = torch.empty(1, 1, dtype=torch.int32, device=gpu)
    wire = S.shard_gather_wire(bank, recv, pref=pref, parts=1)
    rows = torch.empty(bank.cap, bank.row_stride, dtype=torch.float32, device=gpu)
    S.shard_wire_unpack(bank, wire, send, rows, parts=1)
    with pytest.raises(RuntimeError, match="cap_rows"):
        bank.check_flags()
    # gradient records: every valid record carries 1.0 in every element
    wire_g = torch.ones(1, bank.cap_rows * bank.wire_bytes() // 4, dtype=torch.float32,
                        device=gpu).view(torch.uint8)
    before = bank.weight.detach().clone()
    plan = S.owner_plan(bank, recv, bank.part, 1)
    S.owner_apply_wire(bank, plan, wire_g, pref, lr=0.5, parts=1)
    bank.check_flags()
    torch.cuda.synchronize()
    slot_ids = send.view(-1)[:bank.cap].long()  # the distinct ids in slot order
    cols = D + 1 if bank.has_w else D
    for j in range(40):
        r = int(slot_ids[j])
        got, old = bank.weight[r, :D], before[r, :D]
        if j < bank.cap_rows:
            assert torch.equal(got, old - 0.5), j  # one record: gradient 1.0
        else:
            assert torch.equal(got, old), j  # clipped: zero gradient
    untouched = torch.ones(n_rows, dtype=torch.bool, device=gpu)
    untouched[slot_ids[:40]] = False
    assert torch.equal(bank.weight[untouched, :cols], before[untouched, :cols])


def test_sharded_checkpoint_world1_gpu_bit_exact_and_memory_bounded(gpu, tmp_path):
    """Row-sharded checkpoint on the GPU (checkpoint.py): a
    world-1 sharded DeepFM of 26 x 10^6-row bf16 tables (1.66 GB bank) trained one
    step, then ``save_weights`` (the shard streamed device -> host -> file in chunks)
    and ``load_weights`` into a fresh sharded replica and into an unsharded model:
    every row bit-identical to the trained bank, dense entries equal, and the
    unsharded model's own single-file checkpoint loads back into a sharded replica
    bit-identically.  Peak GPU memory above the model's during save and load stays
    below one shard (the whole never exists twice: < 2x the shard in total)."""
    from pytorchrec_amd.embedding import init_bank_
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.model import DeepFM
    from pytorchrec_amd.sharding import ShardComm, sharded_tables
    rows = [1_000_000] * 26
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{i}") for i, n in enumerate(rows)]
    dense = [NumericColumn(f"c_n_I{i}") for i in range(13)]
    label = CategoricalColumnWithIdentity(2, "label")

    def build(sharded, seed):
        mk = lambda: DeepFM(sparse, dense, label, emb_size=16, layers=(64, 32),  # noqa: E731
                            emb_dtype=torch.bfloat16, random_seed=seed, device=gpu)
        if not sharded:
            return mk()
        with sharded_tables(ShardComm(world=1, rank=0), max_batch=512):
            return mk()

    m = build(True, 5)
    init_bank_(m.embeddings, generator=torch.Generator(device=gpu).manual_seed(9))
    m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
    g = torch.Generator().manual_seed(4)
    data = {f"c_c_C{i}": torch.randint(0, n, (512,), generator=g, dtype=torch.int32).to(gpu)
            for i, n in enumerate(rows)}
    for i in range(13):
        data[f"c_n_I{i}"] = torch.rand(512, generator=g).to(gpu)
    data["label"] = (torch.rand(512, generator=g) < 0.25).to(torch.int32).to(gpu)
    m.train_step(data)
    shard_bytes = m.embeddings.weight.numel() * m.embeddings.weight.element_size()
    path = str(tmp_path / "c5like.pt")
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    m.save_weights(path)
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - base < shard_bytes, "save materialised the bank"
    want = m.embeddings.weight.detach().view(torch.int16)
    fresh = build(True, 77)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    fresh.load_weights(path, gpu)
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - base < shard_bytes, "load materialised the bank"
    assert torch.equal(fresh.embeddings.weight.detach().view(torch.int16), want)
    for k, v in m.state_dict().items():
        if k != "embeddings.weight":
            assert torch.equal(fresh.state_dict()[k], v), k
    del fresh
    u = build(False, 78)  # unsharded EmbeddingBank: the same rows at world 1
    u.load_weights(path, gpu)
    assert torch.equal(u.embeddings.weight.detach().view(torch.int16), want)
    single = str(tmp_path / "single.pt")
    u.save_weights(single)  # the reference's single-file format
    del u
    back = build(True, 79)
    back.load_weights(single, gpu)
    assert torch.equal(back.embeddings.weight.detach().view(torch.int16), want)


@pytest.mark.parametrize("quarters,W,B", [(4, 8, 4096), (2, 3, 1000), (4, 1, 4096), (16, 2, 300)])
def test_dedup_bucketize_in_quarters_matches_restatement(gpu, quarters, W, B):
    """mrec_shard_bucketize_dedup_q (ABI 28): `quarters` workgroups per table, each
    taking the ids of its quarter and meeting its siblings once through the scratch
    tickets, give exactly the CPU restatement's quarter-major message and slots, call
    after call (the tickets only grow); Zipf ids with many repeats included."""
    from pytorchrec_amd import sharding as S
    b = S.ShardedEmbeddingBank(ROWS, D, S.ShardComm(world=W, rank=0), with_first_order=True,
                               dtype=torch.bfloat16, max_batch=B, device=gpu)
    b.dedup_quarters = quarters
    for call, zipf in enumerate((False, True, False)):
        ids = _ids(gpu, B, 70 + call, zipf)
        send, pos = S.shard_bucketize_dedup(b, ids)
        ref_send, ref_pos = S.cpu_bucketize_dedup(b, [t.cpu() for t in ids])
        b.check_flags()
        assert torch.equal(send.cpu(), ref_send), (quarters, W, call)
        assert torch.equal(pos.cpu(), ref_pos), (quarters, W, call)
