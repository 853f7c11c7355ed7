"""GPU parity of the embedding kernels (libmrec via ctypes) against the CPU
oracle (oracle/ref.py) and the reference's golden vectors.

Bars (north_star): index gather bit-exact; fp interaction within 1e-5 relative
with the magnitude-aware denominator of SURVEY.md §7 hard part 3; scatter-add
gradients within fp32 reordering tolerance of the fp64 oracle.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def _bank(category_nums, dim, has_w, dtype, update="dense", device="cuda"):
    from pytorchrec_amd import _mrec
    from pytorchrec_amd.embedding import EmbeddingBank
    assert _mrec.available(), "libmrec.so must be built and loadable on the GPU box"
    b = EmbeddingBank(category_nums, dim, with_first_order=has_w, dtype=dtype, update=update,
                      device=device)
    return b


def _fill(bank, tables, ws=None):
    """Write per-table numpy values (fp32 or bf16 bits) into the bank."""
    with torch.no_grad():
        bank.weight.zero_()
        for f, t in enumerate(tables):
            o = bank.row_offset[f]
            if t.dtype == np.uint16:
                tt = torch.from_numpy(t.view(np.int16)).view(torch.bfloat16)
            else:
                tt = torch.from_numpy(t).to(bank.weight.dtype)
            bank.weight[o:o + t.shape[0], :bank.dim] = tt.to(bank.weight.device)
            if ws is not None:
                bank.weight[o:o + t.shape[0], bank.dim] = torch.from_numpy(ws[f]).to(
                    bank.weight.device, bank.weight.dtype)


def _bits(t):
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy().view(np.uint32)


def _wbits(a):
    return a if a.dtype == np.uint16 else np.ascontiguousarray(a, np.float32).view(np.uint32)


def _ids_with_edges(rng, rows, B):
    ids = rng.integers(0, rows, B)
    ids[:4] = [0, rows - 1, 0, rows - 1]
    ids[4:8] = ids[8:12]
    return ids


def _rand_tables(rng, nums, dim, dtype):
    tabs = [(rng.standard_normal((n, dim)) * 0.5).astype(np.float32) for n in nums]
    if dtype == torch.bfloat16:
        tabs = [ref.f32_to_bf16_bits(t) for t in tabs]
    return tabs


def _as_f32(t):
    return ref.bf16_bits_to_f32(t) if t.dtype == np.uint16 else t


# ---------------------------------------------------------------------------
# gather
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gather_golden_g1_bit_exact(gpu, dtype):
    from pytorchrec_amd.embedding import gather
    g = golden("g1_gather.npz")
    table = g["table"] if dtype == torch.float32 else g["table_bf16"]
    want = g["out"] if dtype == torch.float32 else g["out_bf16"]
    bank = _bank([table.shape[0]], table.shape[1], False, dtype)
    _fill(bank, [table])
    ids = torch.from_numpy(g["ids"]).to(gpu)  # int64, as .long() gives
    out = gather(bank, [ids])
    assert np.array_equal(_bits(out), _wbits(want))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("id_dtype", [torch.int32, torch.int64])
def test_gather_multi_table_bit_exact(gpu, dtype, id_dtype):
    from pytorchrec_amd.embedding import gather
    rng = np.random.default_rng(3)
    nums = [int(x) for x in rng.integers(2, 3000, 26)]
    nums[0] = 1  # a one-row table
    D, B = 16, 1000
    tabs = _rand_tables(rng, nums, D, dtype)
    wts = [rng.standard_normal(n).astype(np.float32) for n in nums]
    bank = _bank(nums, D, True, dtype)
    _fill(bank, tabs, wts)
    ids_np = np.stack([_ids_with_edges(rng, n, B) for n in nums], 1)
    ids = [torch.from_numpy(ids_np[:, f]).to(gpu, id_dtype) for f in range(26)]
    out, w = gather(bank, ids, with_w=True)
    want = ref.multi_table_gather(tabs, ids_np).reshape(B, -1)
    assert np.array_equal(_bits(out), _wbits(want))
    wq = [(_as_f32(ref.f32_to_bf16_bits(x)) if dtype == torch.bfloat16 else x) for x in wts]
    want_w = np.stack([wq[f][ids_np[:, f]] for f in range(26)], 1)
    assert np.array_equal(w.detach().cpu().numpy(), want_w)
    # widened / narrowed outputs
    out32 = gather(bank, ids, out_dtype=torch.float32)
    assert np.array_equal(out32.detach().cpu().numpy(), _as_f32(want) if want.dtype == np.uint16 else want)


def test_gather_out_of_range_raises_index_error(gpu):
    from pytorchrec_amd.embedding import gather
    bank = _bank([10, 20], 8, False, torch.float32)
    _fill(bank, [np.ones((10, 8), np.float32), np.ones((20, 8), np.float32)])
    good = torch.tensor([0, 9], device=gpu)
    with pytest.raises(IndexError):
        gather(bank, [good, torch.tensor([0, 20], device=gpu)])
    with pytest.raises(IndexError):
        gather(bank, [torch.tensor([-1, 0], device=gpu), good])
    out = gather(bank, [good, torch.tensor([19, 0], device=gpu)])
    assert torch.all(out == 1)


def test_gather_empty_batch(gpu):
    from pytorchrec_amd.embedding import gather
    bank = _bank([10], 8, False, torch.float32)
    out = gather(bank, [torch.empty(0, dtype=torch.int64, device=gpu)])
    assert out.shape == (0, 8)


# ---------------------------------------------------------------------------
# fused interaction
# ---------------------------------------------------------------------------

def _fm_tol_ok(got, v, want, rtol=1e-5):
    den = np.abs(want) + ref.fm2_magnitude(v)
    return np.all(np.abs(got - want) <= rtol * den + 1e-12), np.max(np.abs(got - want) / den)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_interact_deepfm_stage(gpu, dtype):
    from pytorchrec_amd.embedding import interact
    rng = np.random.default_rng(5)
    nums = [int(x) for x in rng.integers(50, 5000, 26)]
    D, B, ND = 16, 777, 13
    tabs = _rand_tables(rng, nums, D, dtype)
    wts = [(rng.standard_normal(n) * 0.3).astype(np.float32) for n in nums]
    bank = _bank(nums, D, True, dtype)
    _fill(bank, tabs, wts)
    ids_np = np.stack([_ids_with_edges(rng, n, B) for n in nums], 1)
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(26)]
    dense = rng.random((B, ND)).astype(np.float32)
    dense_w = (rng.standard_normal(ND) * 0.1).astype(np.float32)
    bias = np.array([0.25], np.float32)
    x0, logit = interact(bank, ids, torch.from_numpy(dense).to(gpu),
                         torch.from_numpy(dense_w).to(gpu), torch.from_numpy(bias).to(gpu),
                         fm2=True, first_order=True, x0_cols=448, x0_dtype=torch.bfloat16)
    v = _as_f32(ref.multi_table_gather(tabs, ids_np))  # exactly what the kernel reads
    wq = [(_as_f32(ref.f32_to_bf16_bits(x)) if dtype == torch.bfloat16 else x) for x in wts]
    w_g = np.stack([wq[f][ids_np[:, f]] for f in range(26)], 1)
    want = ref.fm2(v) + ref.first_order(w_g, dense, dense_w, bias[0])
    ok, worst = _fm_tol_ok(logit.detach().cpu().numpy().astype(np.float64), v, want)
    assert ok, worst
    # x0 = [v | dense | 0]: embeddings bit-exact in bf16, dense RNE-rounded, pad zero
    x0n = _bits(x0)
    want_v = ref.f32_to_bf16_bits(v.reshape(B, -1))
    assert np.array_equal(x0n[:, :26 * D], want_v)
    assert np.array_equal(x0n[:, 26 * D:26 * D + ND], ref.f32_to_bf16_bits(dense))
    assert np.all(x0n[:, 26 * D + ND:] == 0)


def test_interact_fm_equals_funksvd_golden_g3(gpu):
    """FM over {uid, iid} == FunkSVD.forward (FunkSVD.py:51) — SURVEY G3."""
    from pytorchrec_amd.embedding import interact
    g = golden("g3_funksvd.npz")
    D = g["u_table"].shape[1]
    bank = _bank([g["u_table"].shape[0], g["i_table"].shape[0]], D, False, torch.float32)
    _fill(bank, [g["u_table"], g["i_table"]])
    ids = [torch.from_numpy(g["uid"]).to(gpu), torch.from_numpy(g["iid"]).to(gpu)]
    logit = interact(bank, ids, fm2=True, first_order=False)
    np.testing.assert_allclose(logit.detach().cpu().numpy(), g["prediction"], rtol=1e-5, atol=1e-9)


# ---------------------------------------------------------------------------
# backward
# ---------------------------------------------------------------------------

def test_dense_grad_golden_g2(gpu):
    from pytorchrec_amd.embedding import gather
    g = golden("g2_dense_grad.npz")
    g1 = golden("g1_gather.npz")
    rows = int(g["rows"])
    bank = _bank([rows], g["dy"].shape[1], False, torch.float32, update="dense")
    _fill(bank, [g1["table"]])
    out = gather(bank, [torch.from_numpy(g["ids"]).to(gpu)])
    out.backward(torch.from_numpy(g["dy"]).to(gpu))
    got = bank.weight.grad[:, :bank.dim].detach().cpu().numpy()
    np.testing.assert_allclose(got, g["grad"], rtol=1e-6, atol=1e-7)
    untouched = np.setdiff1d(np.arange(rows), g["ids"])
    assert np.all(got[untouched] == 0)


@pytest.mark.parametrize("zipf", [False, True])
def test_fused_sgd_f32_matches_oracle(gpu, zipf):
    """Row-sparse SGD through the interact backward (dx from the MLP, FM2 and
    first-order grads) == dense SGD on the oracle's dense gradient."""
    from pytorchrec_amd.embedding import interact
    rng = np.random.default_rng(7 + zipf)
    nums = [300, 40, 1, 5000]
    D, B, F = 16, 3000, 4
    tabs = _rand_tables(rng, nums, D, torch.float32)
    wts = [(rng.standard_normal(n) * 0.3).astype(np.float32) for n in nums]
    bank = _bank(nums, D, True, torch.float32, update="sgd")
    bank.use_fused_sgd(lr=0.05)
    _fill(bank, tabs, wts)
    before = bank.weight.detach().clone()
    if zipf:
        ids_np = np.stack([np.minimum(rng.zipf(1.05, B) - 1, n - 1) for n in nums], 1)
    else:
        ids_np = np.stack([rng.integers(0, n, B) for n in nums], 1)
    ids = [torch.from_numpy(ids_np[:, f]).to(gpu) for f in range(F)]
    bias = torch.zeros(1, device=gpu, requires_grad=True)
    x0, logit = interact(bank, ids, bias=bias, fm2=True, first_order=True, x0_cols=F * D,
                         x0_dtype=torch.float32)
    dx0 = rng.standard_normal((B, F * D)).astype(np.float32)
    dlogit = rng.standard_normal(B).astype(np.float32)
    torch.autograd.backward([x0, logit], [torch.from_numpy(dx0).to(gpu),
                                          torch.from_numpy(dlogit).to(gpu)])
    v = ref.multi_table_gather(tabs, ids_np).astype(np.float64)
    gv = dx0.reshape(B, F, D) + ref.fm2_bwd(v, dlogit)
    after = bank.weight.detach().cpu().numpy().astype(np.float64)
    for f in range(F):
        o, n = bank.row_offset[f], nums[f]
        want = ref.sgd_rows(tabs[f], ids_np[:, f], gv[:, f], 0.05)
        want_w = ref.sgd_rows(wts[f][:, None], ids_np[:, f], dlogit[:, None], 0.05)[:, 0]
        got = after[o:o + n]
        scale = np.abs(tabs[f]).max() + 0.05 * np.abs(ref.dense_grad(n, ids_np[:, f], np.abs(gv[:, f]))).max()
        np.testing.assert_allclose(got[:, :D], want, rtol=0, atol=2e-6 * scale)
        np.testing.assert_allclose(got[:, D], want_w, rtol=0, atol=2e-6 * (1 + np.abs(want_w).max()))
        untouched = np.setdiff1d(np.arange(n), ids_np[:, f])
        assert torch.equal(bank.weight[o + untouched].cpu(), before[o + untouched].cpu())
    assert bias.grad is not None and abs(float(bias.grad) - dlogit.sum()) < 1e-3


@pytest.mark.parametrize("sr", [False, True])
def test_fused_sgd_c2_zipf_b4096(gpu, sr):
    """The bench's batch on the C2 bank (26 x 38,462 bf16 rows with the packed
    first-order column) with Zipf(1.05) ids (SURVEY.md §8(d) variant): hot rows take
    hundreds of lookups per step (the apply's segment / hot-row paths).  Fused SGD
    through the interaction backward (dx from the tower, FM2 and first-order
    gradients, duplicates summed: IModel.py:116-125 -> embedding_dense_backward)
    against ref.sgd_rows in fp64: every touched value within 1 bf16 ulp (RNE: the
    one rounding of w - lr g; SR: either neighbour), untouched rows bit-identical."""
    from pytorchrec_amd.embedding import interact
    rng = np.random.default_rng(105)
    F, R, D, B, lr = 26, 38462, 16, 4096, 0.5
    nums = [R] * F
    bank = _bank(nums, D, True, torch.bfloat16, update="sgd")
    bank.use_fused_sgd(lr=lr)
    bank.stochastic_rounding = sr
    bank.check_ids = False
    tabs = _rand_tables(rng, nums, D, torch.bfloat16)
    wts = [ref.bf16_bits_to_f32(ref.f32_to_bf16_bits((rng.standard_normal(R) * 0.3).astype(np.float32)))
           for _ in range(F)]
    _fill(bank, tabs, wts)
    before = bank.weight.detach().clone()
    ids_np = np.stack([np.minimum(rng.zipf(1.05, B) - 1, R - 1) for _ in range(F)], 1)
    assert np.bincount(ids_np[:, 0]).max() > 100  # hot rows present
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(F)]
    x0, logit = interact(bank, ids, fm2=True, first_order=True, x0_cols=F * D,
                         x0_dtype=torch.bfloat16)
    dx0 = ref.bf16_round((rng.standard_normal((B, F * D)) * 0.01).astype(np.float32))
    dlogit = (rng.standard_normal(B) * 0.01).astype(np.float32)
    torch.autograd.backward([x0, logit], [torch.from_numpy(dx0.astype(np.float32)).to(gpu).to(
        torch.bfloat16), torch.from_numpy(dlogit).to(gpu)])
    v = np.stack([_as_f32(tabs[f])[ids_np[:, f]] for f in range(F)], 1).astype(np.float64)
    gv = dx0.reshape(B, F, D) + ref.fm2_bwd(v, dlogit)
    after = _bits(bank.weight)
    for f in range(F):
        o = bank.row_offset[f]
        want = ref.sgd_rows(_as_f32(tabs[f]), ids_np[:, f], gv[:, f], lr)
        want_w = ref.sgd_rows(wts[f][:, None].astype(np.float64), ids_np[:, f], dlogit[:, None],
                              lr)[:, 0]
        got = ref.bf16_bits_to_f32(after[o:o + R, :D + 1]).astype(np.float64)
        touched = np.unique(ids_np[:, f])
        assert np.all(np.abs(got[touched, :D] - want[touched]) <=
                      ref.bf16_ulp(want[touched]) * 1.0001), f
        assert np.all(np.abs(got[touched, D] - want_w[touched]) <=
                      ref.bf16_ulp(want_w[touched]) * 1.0001), f
        untouched = np.setdiff1d(np.arange(R), touched)
        assert torch.equal(bank.weight[o + untouched].cpu(), before[o + untouched].cpu()), f


def test_fused_sgd_bf16_stochastic_rounding_within_one_ulp(gpu):
    from pytorchrec_amd.embedding import gather
    rng = np.random.default_rng(11)
    nums = [2000, 2000]
    D, B = 16, 4096
    tabs = _rand_tables(rng, nums, D, torch.bfloat16)
    bank = _bank(nums, D, False, torch.bfloat16, update="sgd")
    bank.use_fused_sgd(lr=0.1)
    _fill(bank, tabs)
    ids_np = np.stack([np.minimum(rng.zipf(1.2, B) - 1, n - 1) for n in nums], 1)
    ids = [torch.from_numpy(ids_np[:, f]).to(gpu) for f in range(2)]
    out = gather(bank, ids, out_dtype=torch.float32)
    dy = (rng.standard_normal((B, 2 * D)) * 0.01).astype(np.float32)
    out.backward(torch.from_numpy(dy).to(gpu))
    after = _bits(bank.weight)
    for f in range(2):
        o, n = bank.row_offset[f], nums[f]
        want = ref.sgd_rows(_as_f32(tabs[f]), ids_np[:, f], dy[:, f * D:(f + 1) * D], 0.1)
        got = ref.bf16_bits_to_f32(after[o:o + n, :D]).astype(np.float64)
        assert np.all(np.abs(got - want) <= ref.bf16_ulp(want) * 1.0001)


def test_plan_handles_all_duplicates_and_single_row(gpu):
    """Every lookup hits row 0 (one segment of length B, the hot-row path)."""
    from pytorchrec_amd.embedding import gather
    bank = _bank([3], 8, False, torch.float32, update="dense")
    _fill(bank, [np.zeros((3, 8), np.float32)])
    B = 5000
    out = gather(bank, [torch.zeros(B, dtype=torch.int64, device=gpu)])
    dy = torch.ones(B, 8, device=gpu)
    out.backward(dy)
    g = bank.weight.grad[:, :8].detach().cpu().numpy()
    assert np.all(g[0] == B) and np.all(g[1:] == 0)


@pytest.mark.parametrize("B", [1, 777, 4096, 4097, 8192])
def test_dense_grad_bit_exact_ascending_order(gpu, B):
    """Both plans (hash plan for B <= 4096: singles + sorted duplicates; full
    sort above) sum a row's lookups in fp32, ascending sample order: for rows
    hit <= kShortSeg (16) times bitwise equal to a sequential fp32 np.add.at.
    Hot rows use the fixed-order workgroup tree: fp32-reordering tolerance, and
    bitwise reproducible run to run.  Large table (hash path), mid table, and a
    small table (full-sort branch of the hash kernel); Zipf ids so singles,
    short and hot segments all occur."""
    from pytorchrec_amd.embedding import gather
    rng = np.random.default_rng(100 + B)
    nums = [200000, 4096, 50]
    D, F = 8, 3
    bank = _bank(nums, D, False, torch.float32, update="dense")
    _fill(bank, [np.zeros((n, D), np.float32) for n in nums])
    ids_np = np.stack([np.minimum(rng.zipf(1.1, B) - 1, n - 1) if f != 1 else rng.integers(0, n, B)
                       for f, n in enumerate(nums)], 1)
    ids = [torch.from_numpy(ids_np[:, f]).to(gpu) for f in range(F)]
    out = gather(bank, ids, out_dtype=torch.float32)
    dy = rng.standard_normal((B, F * D)).astype(np.float32)
    out.backward(torch.from_numpy(dy).to(gpu))
    got = bank.weight.grad[:, :D].detach().cpu().numpy().copy()
    bank.weight.grad = None
    gather(bank, ids, out_dtype=torch.float32).backward(torch.from_numpy(dy).to(gpu))
    assert np.array_equal(got.view(np.uint32), bank.weight.grad[:, :D].cpu().numpy().view(np.uint32))
    for f in range(F):
        o, n = bank.row_offset[f], nums[f]
        want = np.zeros((n, D), np.float32)
        np.add.at(want, ids_np[:, f], dy[:, f * D:(f + 1) * D])  # sequential fp32, index order
        cnt = np.bincount(ids_np[:, f], minlength=n)
        short = cnt <= 16
        assert np.array_equal(got[o:o + n][short].view(np.uint32), want[short].view(np.uint32)), f
        mag = ref.dense_grad(n, ids_np[:, f], np.abs(dy[:, f * D:(f + 1) * D]))
        assert np.all(np.abs(got[o:o + n] - want) <= 1e-6 * mag + 1e-30), f


def _large_case(rng, nums, B):
    """ids with every segment kind: rows hit once, 2..16 times (register sort),
    17..2048 (one fixed-point chunk), and one row per table hit > 2048 times
    (several chunks), plus a DIN-like PAD row 0."""
    cols = []
    for n in nums:
        x = rng.integers(0, n, B)
        x[rng.random(B) < 0.3] = 0                      # hot PAD row: ~0.3 B lookups
        if n > 64:
            x[rng.random(B) < 0.05] = rng.integers(1, 40, 1)[0]  # a second hot row
        cols.append(x)
    return np.stack(cols, 1)


@pytest.mark.parametrize("B,nums", [(20000, [63002, 802]), (9000, [5, 70001, 1])])
def test_backward_large_batch_dense_grad(gpu, B, nums):
    """B > MREC_BWD_MAX_BATCH: device-wide plan + ONE accumulation per row
    (emb_bwd_large.hip).  Rows hit <= 16 times: bitwise equal to sequential fp32
    np.add.at (ascending sample order); hotter rows (fixed-point sums): within fp32
    rounding of the fp64 oracle; bitwise reproducible run to run."""
    from pytorchrec_amd.embedding import gather
    rng = np.random.default_rng(B)
    D, F = 16, len(nums)
    bank = _bank(nums, D, False, torch.float32, update="dense")
    _fill(bank, [np.zeros((n, D), np.float32) for n in nums])
    ids_np = _large_case(rng, nums, B)
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(F)]
    dy = (rng.standard_normal((B, F * D)) * 1e-3).astype(np.float32)
    gather(bank, ids, out_dtype=torch.float32).backward(torch.from_numpy(dy).to(gpu))
    got = bank.weight.grad[:, :D].detach().cpu().numpy().copy()
    bank.weight.grad = None
    gather(bank, ids, out_dtype=torch.float32).backward(torch.from_numpy(dy).to(gpu))
    assert np.array_equal(got.view(np.uint32), bank.weight.grad[:, :D].cpu().numpy().view(np.uint32))
    for f in range(F):
        o, n = bank.row_offset[f], nums[f]
        seq = np.zeros((n, D), np.float32)
        np.add.at(seq, ids_np[:, f], dy[:, f * D:(f + 1) * D])
        cnt = np.bincount(ids_np[:, f], minlength=n)
        short = cnt <= 16
        assert np.array_equal(got[o:o + n][short].view(np.uint32), seq[short].view(np.uint32)), f
        want = ref.dense_grad(n, ids_np[:, f], dy[:, f * D:(f + 1) * D].astype(np.float64))
        mag = ref.dense_grad(n, ids_np[:, f], np.abs(dy[:, f * D:(f + 1) * D]).astype(np.float64))
        # hot rows (fixed point): one fp32 rounding of the exact sum (+ 2^-45 of the
        # largest term per lookup)
        hot = ~short
        assert hot.any()
        err = np.abs(got[o:o + n][hot] - want[hot])
        assert np.all(err <= 2 ** -24 * np.abs(want[hot]) + 1e-12 * mag[hot] + 1e-30), f


@pytest.mark.parametrize("B,hot", [(20000, 0.3), (150000, 0.7)])
@pytest.mark.parametrize("update", ["dense", "sgd"])
def test_bucketed_plan_matches_atomic_plan(gpu, B, hot, update, monkeypatch):
    """Batches of <= 2M lookups take the bucketed plan (lookups partitioned by a hash
    of their row, one workgroup per bucket groups its rows in LDS), fused with the
    updates (mrec_emb_bwd_large_fused) or as the plan / apply pair.  Every path sums
    a row's lookups with the same arithmetic (ascending sample order up to 16,
    order-free fixed point beyond), so the results are bitwise those of the atomic
    plan (MREC_LG_ATOMIC_PLAN=1) -- also across many chunks (B=150000: 37 chunks)
    and for a row hit > 2^16 times (2048+: the chunked kernels)."""
    from pytorchrec_amd import embedding as E
    rng = np.random.default_rng(B)
    nums, D = [63002, 802], 16
    ids_np = np.stack([rng.integers(0, n, B) for n in nums], 1)
    ids_np[rng.random(B) < hot, 0] = 0
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(2)]
    dy = torch.from_numpy((rng.standard_normal((B, 2 * D)) * 1e-3).astype(np.float32)).to(gpu)
    dtype = torch.float32 if update == "dense" else torch.bfloat16
    tabs = [(rng.standard_normal((n, D)) * 0.1).astype(np.float32) for n in nums]
    got = {}
    for path in ("fused", "pair", "atomic"):
        monkeypatch.setattr(E, "LARGE_FUSED", path == "fused")
        if path == "atomic":
            monkeypatch.setenv("MREC_LG_ATOMIC_PLAN", "1")
        bank = _bank(nums, D, False, dtype, update=update)
        if update == "sgd":
            bank.use_fused_sgd(0.5)
            bank.stochastic_rounding = False
        _fill(bank, tabs)
        E.gather(bank, ids, out_dtype=torch.float32).backward(dy)
        res = bank.weight.grad if update == "dense" else bank.weight
        got[path] = _bits(res[:, :D])
    monkeypatch.delenv("MREC_LG_ATOMIC_PLAN")
    assert (ids_np[:, 0] == 0).sum() > (1 << 16) or B < 100000
    assert np.array_equal(got["fused"], got["atomic"])
    assert np.array_equal(got["pair"], got["atomic"])
    if update == "dense":
        want = ref.dense_grad(nums[0], ids_np[:, 0], dy[:, :D].cpu().numpy().astype(np.float64))
        assert np.allclose(got["fused"].view(np.float32)[:nums[0]], want, rtol=1e-5, atol=1e-7)


def test_huge_segment_wait_timeout_raises_and_leaves_rows_untouched(gpu, monkeypatch):
    """The fused large-batch path sums rows hit > 2048 times in one launch of three
    dependent phases (max |g|, fixed-point chunk sums, the update) whose work items
    are dequeued in phase order: no co-residency is assumed, so a phase wait always
    ends.  Its waits are still bounded; MREC_LG_HUGE_TEST_STALL=1 (test-only) makes
    them unreachable.  Then the backward raises RuntimeError (the workspace's sticky
    error word, read by EmbeddingBank.check_flags), the huge rows keep their bits
    (never an update from partial sums), every other row gets exactly the update of
    a normal run, and the next normal call is clean and bitwise equal to the atomic
    plan."""
    from pytorchrec_amd import embedding as E
    rng = np.random.default_rng(77)
    nums, D, B = [63002, 802], 16, 20000
    ids_np = np.stack([rng.integers(0, n, B) for n in nums], 1)
    ids_np[rng.random(B) < 0.3, 0] = 5   # row 5 of table 0: ~6000 lookups (huge)
    ids_np[rng.random(B) < 0.2, 1] = 3   # row 3 of table 1: ~4000 lookups (huge)
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(2)]
    dy = torch.from_numpy((rng.standard_normal((B, 2 * D)) * 1e-2).astype(np.float32)).to(gpu)
    tabs = [ref.f32_to_bf16_bits((rng.standard_normal((n, D)) * 0.1).astype(np.float32))
            for n in nums]
    def run(stall, atomic=False):
        if stall:
            monkeypatch.setenv("MREC_LG_HUGE_TEST_STALL", "1")
        if atomic:
            monkeypatch.setenv("MREC_LG_ATOMIC_PLAN", "1")
        bank = _bank(nums, D, False, torch.bfloat16, update="sgd")
        bank.use_fused_sgd(0.5)
        bank.stochastic_rounding = False
        _fill(bank, tabs)
        b0 = _bits(bank.weight[:, :D])
        out = E.gather(bank, ids, out_dtype=torch.float32)
        err = None
        try:
            out.backward(dy)
            torch.cuda.synchronize()
        except RuntimeError as e:
            err = e
        monkeypatch.delenv("MREC_LG_HUGE_TEST_STALL", raising=False)
        monkeypatch.delenv("MREC_LG_ATOMIC_PLAN", raising=False)
        return bank, b0, _bits(bank.weight[:, :D]), err

    monkeypatch.setattr(E, "LARGE_FUSED", True)
    bank_s, before, stalled, err = run(True)
    huge = [bank_s.row_offset[0] + 5, bank_s.row_offset[1] + 3]
    assert err is not None and "huge-segment" in str(err), err
    bank_s.check_flags()  # the word was cleared by the raise
    _, _, normal, err2 = run(False)
    assert err2 is None
    _, _, atomic, _ = run(False, atomic=True)
    assert np.array_equal(normal, atomic)
    for r in huge:
        assert np.array_equal(stalled[r], before[r]), r      # untouched, not half-updated
        assert not np.array_equal(normal[r], before[r]), r   # a normal run does move them
    keep = np.ones(stalled.shape[0], bool)
    keep[huge] = False
    assert np.array_equal(stalled[keep], normal[keep])


def test_backward_large_batch_sgd_one_update_per_row(gpu):
    """Fused SGD at B > MREC_BWD_MAX_BATCH updates every touched row exactly once:
    new = RNE_bf16(old - lr * sum g), equal to the fp64 oracle's sum rounded once
    (within 1 bf16 ulp, where the fp32 sum may straddle a rounding boundary);
    untouched rows keep their bits."""
    from pytorchrec_amd.embedding import gather
    rng = np.random.default_rng(3)
    nums, D, B, lr = [63002, 802], 16, 30000, 0.5
    bank = _bank(nums, D, False, torch.bfloat16, update="sgd")
    bank.use_fused_sgd(lr)
    bank.stochastic_rounding = False
    tabs = [ref.f32_to_bf16_bits(rng.standard_normal((n, D)).astype(np.float32) * 0.1)
            for n in nums]
    _fill(bank, tabs)
    before = _as_f32(_bits(bank.weight[:, :D]))
    ids_np = _large_case(rng, nums, B)
    ids = [torch.from_numpy(ids_np[:, f].astype(np.int32)).to(gpu) for f in range(2)]
    dy = (rng.standard_normal((B, 2 * D)) * 1e-2).astype(np.float32)
    out = gather(bank, ids, out_dtype=torch.float32)
    out.backward(torch.from_numpy(dy).to(gpu))
    after = _as_f32(_bits(bank.weight[:, :D]))
    for f in range(2):
        o, n = bank.row_offset[f], nums[f]
        g = ref.dense_grad(n, ids_np[:, f], dy[:, f * D:(f + 1) * D].astype(np.float64))
        want = before[o:o + n].astype(np.float64) - lr * g
        touched = np.bincount(ids_np[:, f], minlength=n) > 0
        assert np.array_equal(after[o:o + n][~touched], before[o:o + n][~touched])
        err = np.abs(after[o:o + n][touched] - want[touched])
        assert np.all(err <= ref.bf16_ulp(want[touched]) * 1.01), f


def test_fm2_dense_kernel(gpu):
    from pytorchrec_amd.embedding import fm2_dense
    rng = np.random.default_rng(17)
    v = rng.standard_normal((300, 13, 24)).astype(np.float32)
    vt = torch.from_numpy(v).to(gpu).requires_grad_()
    y = fm2_dense(vt)
    ok, worst = _fm_tol_ok(y.detach().cpu().numpy().astype(np.float64), v, ref.fm2(v))
    assert ok, worst
    dy = rng.standard_normal(300).astype(np.float32)
    y.backward(torch.from_numpy(dy).to(gpu))
    np.testing.assert_allclose(vt.grad.detach().cpu().numpy(), ref.fm2_bwd(v, dy), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("rows", [7, 5000, 200000])
def test_plan_inside_interaction_launch_matches_standalone(gpu, rows):
    """The (table, bucket) hash plan run by leading workgroups of the interaction
    launch (mrec_interact_fwd_ex) drives the same updates as the standalone plan
    kernel: bitwise, on hot Zipf rows, uniform rows and a table of 7 rows (every
    row repeated: direct-indexed slots); and a plan job inside a GEMM launch is
    refused (ABI 12)."""
    import ctypes
    from pytorchrec_amd import _mrec
    rng = np.random.default_rng(rows)
    B, F, D = 4096, 3, 16
    ids_np = np.stack([np.minimum(rng.zipf(1.2, B) - 1, rows - 1), rng.integers(0, rows, B),
                       rng.integers(0, max(1, rows // 3), B)], 1).astype(np.int64)
    ids = [torch.from_numpy(np.ascontiguousarray(ids_np[:, f])).to(gpu) for f in range(F)]
    dy = torch.from_numpy(rng.standard_normal((B, F * D)).astype(np.float32)).to(gpu)
    results = []
    for fused in (False, True):
        bank = _bank([rows] * F, D, False, torch.float32, update="dense")
        _fill(bank, [np.zeros((rows, D), np.float32)] * F)
        idd = _mrec.IdsDesc(ids)
        wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, B)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=gpu)
        if fused:
            job = _mrec.PlanJob(ctypes.pointer(bank.desc().struct), ctypes.pointer(idd.struct), B,
                                ws.data_ptr(), wsb, None, None)
            bank.desc().ref()
            logit = torch.empty(B, device=gpu)
            _mrec.call("mrec_interact_fwd_ex", bank.desc().ref(), idd.ref(), B, None, 0, 0, None,
                       None, 0, None, _mrec.F32, 0, 0, logit.data_ptr(), None, None,
                       ctypes.byref(job), _mrec.stream_handle())
            with pytest.raises(_mrec.MrecError):
                _mrec.call("mrec_gemm_multi_ex", 0, None, ctypes.byref(job), None,
                           _mrec.stream_handle())
        else:
            _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), idd.ref(), B, ws.data_ptr(), wsb,
                       None, None, _mrec.stream_handle())
        grad = torch.zeros_like(bank.weight)
        _mrec.call("mrec_emb_bwd_apply", bank.desc().ref(), B, ws.data_ptr(), wsb, dy.data_ptr(),
                   _mrec.F32, dy.stride(0), None, None, None, _mrec.F32, 0, None,
                   _mrec.BWD_DENSE_GRAD, 0.0, 0, None, grad.data_ptr(), _mrec.stream_handle())
        results.append(grad[:, :D].cpu().numpy())
    assert np.array_equal(results[0].view(np.uint32), results[1].view(np.uint32))
    want = ref.dense_grad(rows, ids_np[:, 0], dy[:, :D].cpu().numpy())
    np.testing.assert_allclose(results[1][:rows], want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("threads,slots", [(1024, 8192), (512, 8192), (256, 8192), (512, 4096)])
def test_plan_body_instantiations_match_standalone(gpu, threads, slots):
    """Every workgroup size / slot count the hash-plan body (emb_plan.h
    plan_hash_body) is compiled for -- the production 1024 / 8192 and the
    diagnostic 512 / 8192, 256 / 8192, 512 / 4096 (batches <= 4096) of
    mrec_diag_plan_hash_variant -- leaves a workspace that drives
    mrec_emb_bwd_apply to the standalone plan's dense gradient, bitwise (VERDICT
    r04: the 512-thread body).  Cases: the r04 fault's shape (B = 1000, 5,000 rows per
    table), direct-indexed slots (7 rows), Zipf hot rows and uniform ids at B = 4096,
    a padded exchange view (B = 8192 entries, half of them -1)."""
    import ctypes
    from pytorchrec_amd import _mrec
    fn = _mrec.lib().mrec_diag_plan_hash_variant  # diagnostics: not in mrec.h
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(_mrec.TableBank), ctypes.POINTER(_mrec.Ids), ctypes.c_int64,
                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                   ctypes.c_void_p, ctypes.c_void_p]
    D = 16
    cases = [(1000, 5000, False), (4096, 7, False), (4096, 100000, False), (8192, 30000, True)]
    for B, rows, padded in cases:
        if slots < 8192 and B > 4096:
            continue
        rng = np.random.default_rng(B + rows)
        F = 3
        ids_np = np.stack([np.minimum(rng.zipf(1.2, B) - 1, rows - 1), rng.integers(0, rows, B),
                           rng.integers(0, max(1, rows // 3), B)], 1).astype(np.int64)
        if padded:
            ids_np[rng.random((B, F)) < 0.5] = -1
        ids = [torch.from_numpy(np.ascontiguousarray(ids_np[:, f])).to(gpu) for f in range(F)]
        dy = torch.from_numpy(rng.standard_normal((B, F * D)).astype(np.float32)).to(gpu)
        g_occ = dy[:, :D].contiguous()
        results = []
        for variant in (False, True):
            bank = _bank([rows] * F, D, False, torch.float32, update="dense")
            _fill(bank, [np.zeros((rows, D), np.float32)] * F)
            idd = _mrec.IdsDesc(ids, pad_negative=padded)
            wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, B)
            ws = torch.zeros(wsb, dtype=torch.uint8, device=gpu)
            oob = torch.zeros(1, dtype=torch.int32, device=gpu)
            if variant:
                _mrec.call("mrec_diag_plan_hash_variant", bank.desc().ref(), idd.ref(), B,
                           ws.data_ptr(), wsb, threads, slots, oob.data_ptr(), _mrec.stream_handle())
            else:
                _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), idd.ref(), B, ws.data_ptr(), wsb,
                           oob.data_ptr(), None, _mrec.stream_handle())
            grad = torch.zeros_like(bank.weight)
            if padded and B > 4096:
                # r5b: a padded plan past 4096 entries wrote the hash layout; the plain
                # apply would read it as the sorted one (silently wrong gradients in r05).
                # ABI 28 refuses the pair before launching anything (mrec.h layout rule).
                with pytest.raises(_mrec.MrecError, match="layout mismatch"):
                    _mrec.call("mrec_emb_bwd_apply", bank.desc().ref(), B, ws.data_ptr(), wsb,
                               dy.data_ptr(), _mrec.F32, dy.stride(0), None, None, None,
                               _mrec.F32, 0, None, _mrec.BWD_DENSE_GRAD, 0.0, 0, None,
                               grad.data_ptr(), _mrec.stream_handle())
                torch.cuda.synchronize()
                assert not grad.any(), "a refused apply must not launch"
            if padded:  # an exchange view's apply: the per-entry gradients given (fp32 [B, 16])
                _mrec.call("mrec_emb_bwd_apply_given", bank.desc().ref(), B, ws.data_ptr(), wsb,
                           None, _mrec.F32, 0, None, None, None, _mrec.F32, 0, None, g_occ.data_ptr(),
                           D, 0, 0, _mrec.BWD_DENSE_GRAD, 0.0, 0, None, grad.data_ptr(), 0, None,
                           _mrec.stream_handle())
            else:
                _mrec.call("mrec_emb_bwd_apply", bank.desc().ref(), B, ws.data_ptr(), wsb,
                           dy.data_ptr(), _mrec.F32, dy.stride(0), None, None, None, _mrec.F32, 0,
                           None, _mrec.BWD_DENSE_GRAD, 0.0, 0, None, grad.data_ptr(),
                           _mrec.stream_handle())
            torch.cuda.synchronize()
            assert int(oob.item()) == 0
            results.append(grad[:, :D].cpu().numpy())
        assert np.array_equal(results[0].view(np.uint32), results[1].view(np.uint32)), (B, rows)
        want = ref.dense_grad(rows + 1, np.where(ids_np[:, 0] < 0, rows, ids_np[:, 0]),
                              dy[:, :D].cpu().numpy())[:rows]  # (row `rows`: the padding)
        np.testing.assert_allclose(results[1][:rows], want, rtol=1e-5, atol=1e-5)
