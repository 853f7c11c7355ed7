"""Columnar batch feed (pytorchrec_amd/loader.py).

The loader must hand the model exactly the batches the reference's per-sample
path would build (SimpleDataReader.py:323-331 + default_collate, IModel.py:183-190):
same keys, same rows in the same order, ragged last batch, seeded shuffles.
CPU tests check the packing and the IModel.fit integration; the GPU test checks
the pipelined H2D path bit-for-bit and a DeepFM trained through it against the
same model trained on resident batches.
"""
import numpy as np
import pytest
import torch

from pytorchrec_amd.loader import ColumnarDataset, ColumnarLoader

F_ROWS = [50, 7, 129]
N_DENSE = 3


def _columns(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    cols = {f"c_c_C{i}": torch.randint(0, r, (n,), generator=g, dtype=torch.int64)
            for i, r in enumerate(F_ROWS)}
    for j in range(N_DENSE):
        cols[f"c_n_I{j}"] = torch.rand(n, generator=g, dtype=torch.float64)
    cols["label"] = (torch.rand(n, generator=g) < 0.3).to(torch.int32)
    cols["pos_his"] = torch.randint(0, 9, (n, 5), generator=g, dtype=torch.int32)
    return cols


def _dataset(n, seed=0):
    return ColumnarDataset(_columns(n, seed), dense_group=[f"c_n_I{j}" for j in range(N_DENSE)])


def _expected(cols, idx):
    out = {}
    for k, v in cols.items():
        v = v[idx]
        if v.is_floating_point():
            v = v.float()
        elif v.dtype == torch.int64:
            v = v.to(torch.int32)
        out[k] = v
    return out


@pytest.mark.parametrize("n,batch,drop_last", [(100, 32, False), (100, 32, True), (64, 64, False),
                                               (5, 8, False), (0, 8, False)])
def test_sequential_batches_match_rows(n, batch, drop_last):
    cols = _columns(n)
    ld = ColumnarLoader(_dataset(n), batch, drop_last=drop_last)
    got = list(ld)
    nb = n // batch if drop_last else -(-n // batch)
    assert len(got) == len(ld) == nb
    for j, b in enumerate(got):
        lo, hi = j * batch, min(n, (j + 1) * batch)
        want = _expected(cols, torch.arange(lo, hi))
        for k, v in want.items():
            assert b[k].dtype == v.dtype, k
            assert torch.equal(b[k], v), (j, k)
        dense = torch.stack([want[f"c_n_I{i}"] for i in range(N_DENSE)], 1)
        assert torch.equal(b["__dense__"], dense)
        assert b["c_c_C0"].is_contiguous() and b["__dense__"].is_contiguous()


def test_shuffle_is_a_seeded_permutation_per_epoch():
    n, batch = 103, 16
    cols = _columns(n)
    ld = ColumnarLoader(_dataset(n), batch, shuffle=True, seed=5)
    epochs = []
    for e in range(2):
        order = torch.randperm(n, generator=torch.Generator().manual_seed(5 + e))
        got = torch.cat([b["c_c_C2"].clone() for b in ld])
        assert torch.equal(got, cols["c_c_C2"][order].to(torch.int32))
        epochs.append(got)
    assert not torch.equal(epochs[0], epochs[1])


def test_dataset_getitem_is_the_reference_sample_dict():
    cols = _columns(10)
    ds = _dataset(10)
    s = ds[3]
    assert set(s) == set(cols)
    assert int(s["c_c_C1"]) == int(cols["c_c_C1"][3])
    assert float(s["c_n_I2"]) == float(cols["c_n_I2"][3].float())
    with pytest.raises(ValueError):
        ColumnarDataset({"a": np.zeros(3), "b": np.zeros(4)})
    with pytest.raises(ValueError):
        ColumnarDataset({"a": np.zeros(3, np.int64)}, dense_group=["a"])


def test_copy_mode_is_validated():
    with pytest.raises(ValueError):
        ColumnarLoader(_dataset(4), 2, copy="memcpy")


def test_int64_ids_beyond_int32_stay_int64():
    ds = ColumnarDataset({"c_c_big": np.array([0, 1 << 40, 3], np.int64)})
    b = next(iter(ColumnarLoader(ds, 4)))
    assert b["c_c_big"].dtype == torch.int64 and int(b["c_c_big"][1]) == 1 << 40


def _model(device=None):
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    sparse = [CategoricalColumnWithIdentity(r, f"c_c_C{i}") for i, r in enumerate(F_ROWS)]
    dense = [NumericColumn(f"c_n_I{j}") for j in range(N_DENSE)]
    label = CategoricalColumnWithIdentity(2, "label")
    kw = {} if device is None else {"device": device}
    return DeepFM(sparse, dense, label, emb_size=8, layers=(16, 8), random_seed=7, **kw)


def test_fit_through_columnar_loader_equals_fit_through_dataloader():
    """IModel.fit on a ColumnarDataset (columnar loader) trains exactly like fit on
    the reference's per-sample dataset (DataLoader + default_collate)."""
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    from pytorchrec_amd.metrics import AUC
    n = 200
    cols = _columns(n, seed=3)
    cols.pop("pos_his")

    class Rows(torch.utils.data.Dataset):
        def __len__(self):
            return n

        def __getitem__(self, i):
            return {k: (v[i].float() if v.is_floating_point() else v[i]) for k, v in cols.items()}

    hist = []
    for ds in (Rows(), ColumnarDataset(cols, dense_group=[f"c_n_I{j}" for j in range(N_DENSE)])):
        m = _model()
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [AUC()],
                  torch.device("cpu"))
        hist.append(m.fit(ds, 64, 2, dev_dataset=ds, verbose=0, shuffle=False))
        hist.append({k: v.detach().clone() for k, v in m.state_dict().items()})
    for a, b in zip(hist[0], hist[2]):
        assert a.keys() == b.keys()
        for k in a:
            assert abs(a[k] - b[k]) <= 1e-6 * max(1.0, abs(a[k])), k
    for k in hist[1]:
        torch.testing.assert_close(hist[1][k], hist[3][k], rtol=1e-6, atol=1e-7, msg=k)


def test_prepare_epoch_refused_while_iterating():
    """The host buffer holds the epoch being iterated: repacking it mid-epoch would
    duplicate / drop samples, so it raises; a finished or closed
    iteration releases it."""
    ld = ColumnarLoader(_dataset(100), 32, shuffle=True)
    it = iter(ld)
    next(it)
    with pytest.raises(RuntimeError, match="being iterated"):
        ld.prepare_epoch()
    it.close()
    ld.prepare_epoch()
    assert len(list(ld)) == 4


@pytest.mark.gpu
def test_gpu_pipelined_batches_bit_exact_and_training_matches_resident(gpu):
    n, batch = 1000, 128
    cols = _columns(n, seed=1)
    ds = _dataset(n, seed=1)
    for copy in ("kernel", "dma", "side"):
        _check_pipelined(ColumnarLoader(ds, batch, device=gpu, shuffle=True, seed=11, depth=2,
                                        copy=copy), cols, n, batch)
    for copy in ("kernel", "dma"):
        _check_back_to_back_epochs(ds, cols, n, batch, gpu, copy)
    _check_training(cols, n, batch, gpu)
    # the stage kernel refuses pageable host memory instead of faulting on it
    from pytorchrec_amd import _mrec
    d = torch.empty(64, dtype=torch.uint8, device=gpu)
    with pytest.raises(Exception, match="pinned"):
        _mrec.call("mrec_batch_stage", d.data_ptr(), torch.zeros(64, dtype=torch.uint8).data_ptr(),
                   64, _mrec.stream_handle(gpu))


def _check_pipelined(ld, cols, n, batch):
    order = torch.randperm(n, generator=torch.Generator().manual_seed(11))
    seen = []
    for j, b in enumerate(ld):
        idx = order[j * batch:(j + 1) * batch]
        want = _expected(cols, idx)
        for k, v in want.items():
            assert torch.equal(b[k].cpu(), v), (j, k)
        seen.append(b["c_c_C0"].clone())  # before the slot is refilled
        # a slow consumer: the refill of this slot must wait for this kernel
        torch.cuda._sleep(2_000_000)
        assert torch.equal(b["c_c_C0"].cpu(), want["c_c_C0"]), j
    assert len(seen) == len(ld) == 8


def _check_back_to_back_epochs(ds, cols, n, batch, gpu, copy):
    """Two shuffled epochs with no host sync between them behind a slow consumer:
    packing epoch 2 must wait for epoch 1's last enqueued copies, which still read
    the host buffer."""
    ld = ColumnarLoader(ds, batch, device=gpu, shuffle=True, seed=21, depth=3, copy=copy)
    got = []
    for _ in range(2):
        for b in ld:
            torch.cuda._sleep(3_000_000)
            got.append(b["c_c_C1"].clone())
    torch.cuda.synchronize()
    for e in range(2):
        order = torch.randperm(n, generator=torch.Generator().manual_seed(21 + e))
        for j in range(len(ld)):
            want = _expected(cols, order[j * batch:(j + 1) * batch])["c_c_C1"]
            assert torch.equal(got[e * len(ld) + j].cpu(), want), (copy, e, j)


def _check_training(cols, n, batch, gpu):
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    # DeepFM trained through the loader == trained on the same batches made resident
    cols.pop("pos_his")
    cds = ColumnarDataset(cols, dense_group=[f"c_n_I{j}" for j in range(N_DENSE)])
    losses = []
    for via_loader in (True, False):
        m = _model(device=gpu)
        m.compile(torch.optim.SGD(m.get_parameters(), lr=0.05), BCEWithLogitsLoss(), [], gpu)
        run = []
        if via_loader:
            for b in ColumnarLoader(cds, batch, device=gpu):
                run.append(float(m.train_step(b)["loss"].detach()))
        else:
            for j in range(-(-n // batch)):
                sl = slice(j * batch, (j + 1) * batch)
                b = {k: v[sl].to(gpu) for k, v in _expected(cols, torch.arange(n)).items()}
                b["__dense__"] = torch.stack([b[f"c_n_I{i}"] for i in range(N_DENSE)], 1)
                run.append(float(m.train_step(b)["loss"].detach()))
        losses.append(run)
        losses.append(m.state_dict())
    assert losses[0] == losses[2]
    for k in losses[1]:
        assert torch.equal(losses[1][k], losses[3][k]), k


@pytest.mark.gpu
def test_gpu_graph_epochs_stage_on_a_branch_bit_exact(gpu):
    """ColumnarLoader.capture_steps: one HIP graph of ``depth`` steps, the H2D copy of
    the batch depth - 1 ahead on a branch beside each step (mrec_batch_stage_cursor,
    device cursor): over two shuffled epochs every step sees exactly its batch, with
    a slow step (the copy of the next batches must not overtake it)."""
    n, batch, depth = 1536, 128, 4  # 12 batches: 3 replays per epoch
    cols = _columns(n, seed=3)
    ds = _dataset(n, seed=3)
    ld = ColumnarLoader(ds, batch, device=gpu, shuffle=True, seed=31, depth=depth)
    seen = torch.zeros(depth, batch, dtype=torch.int32, device=gpu)
    dense = torch.zeros(depth, batch, ds.dense.shape[1], dtype=torch.float32, device=gpu)
    calls = [0]

    def step(b):
        j = calls[0] % depth
        calls[0] += 1
        torch.cuda._sleep(1_000_000)
        seen[j].copy_(b["c_c_C0"])
        dense[j].copy_(b["__dense__"])

    for s, _ in ld.iter_slots():  # eager warm-up epoch
        step(ld.slot_views(s))
    ge = ld.capture_steps(step)
    for e in range(2):
        order = torch.randperm(n, generator=torch.Generator().manual_seed(31 + 1 + e))
        for first in ge.replays():
            torch.cuda.synchronize()
            for j in range(depth):
                want = _expected(cols, order[(first + j) * batch:(first + j + 1) * batch])
                assert torch.equal(seen[j].cpu(), want["c_c_C0"]), (e, first, j)
                wd = torch.stack([want[f"c_n_I{k}"] for k in range(N_DENSE)], 1)
                assert torch.equal(dense[j].cpu(), wd), (e, first, j)


@pytest.mark.parametrize("batch", [32, 130, 4096])
def test_narrow_record_widened_equals_the_batch(batch):
    """ABI 29: a kernel-copied GPU loader packs the leading int32 [N] columns whose
    values fit 16 bits (ids, labels) as 16-bit values in the host record and the copy
    widens them into the device slot (mrec_feed_job.widen_bytes).  Restated on the
    CPU: widening the host record's prefix 1:2 (zero-extended) and moving the rest
    by widen_bytes gives a slot whose views are exactly the batch; ids of 65,535 and
    a column past 16 bits stay correct (the latter is not narrowed)."""
    from pytorchrec_amd.loader import PackedLayout
    n = batch + 7
    cols = _columns(n, seed=5)
    cols["c_c_C0"][:3] = torch.tensor([65535, 32768, 0])  # the 16-bit extremes
    cols["c_c_big"] = torch.randint(0, 1 << 20, (n,), dtype=torch.int64)
    ds = ColumnarDataset(cols, dense_group=[f"c_n_I{j}" for j in range(N_DENSE)])
    lay = PackedLayout(ds, batch, narrow=True)
    wide = PackedLayout(ds, batch, narrow=False)
    assert 0 < lay.widen_bytes and lay.widen_bytes % 16 == 0
    assert lay.record_bytes + lay.widen_bytes == lay.slot_bytes
    assert lay.record_bytes <= wide.slot_bytes
    host = torch.zeros(1, lay.record_bytes, dtype=torch.uint8)
    lay.pack(ds, None, host, 1)
    h = host[0].numpy()
    w = lay.widen_bytes
    slot = np.zeros(lay.slot_bytes, dtype=np.uint8)
    slot[:2 * w].view(np.int32)[:] = h[:w].view(np.uint16).astype(np.int32)
    slot[2 * w:] = h[w:]
    got = lay.views(torch.from_numpy(slot), batch)
    want = _expected(cols, torch.arange(batch))
    for k, v in want.items():
        if k.startswith("c_n_I"):
            continue
        assert torch.equal(got[k], v), k
    narrowed = [name for name, *_, nar in lay.segments if nar]
    assert "c_c_C0" in narrowed and "c_c_big" not in narrowed
