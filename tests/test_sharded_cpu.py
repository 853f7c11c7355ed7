"""Row-sharded tables + data-parallel dense tower over world_size 2 (gloo, CPU).

The N>1 path of SURVEY.md §8e, run as two processes on the CPU with the same
exchange protocol (bucketize -> all_to_all ids -> owner gather -> all_to_all rows;
backward: slot gradients -> reverse all_to_all -> owner SGD / W; dense grads
all-reduced and averaged).  Checked against ONE process training the unsharded
model on the concatenation of both ranks' batches: same loss, same dense
parameters, and every shard equal to its rows of the single-process tables.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

from conftest import ROOT

F_ROWS = [50, 7, 129, 1]   # includes a single-row table (empty on rank 1)
DIM, N_DENSE, B, LAYERS, LR = 8, 3, 32, (16, 8), 0.05


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _columns():
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{i}") for i, n in enumerate(F_ROWS)]
    dense = [NumericColumn(f"c_n_I{i}") for i in range(N_DENSE)]
    label = CategoricalColumnWithIdentity(2, "label")
    return sparse, dense, label


def _batch(seed, n):
    g = torch.Generator().manual_seed(seed)
    data = {f"c_c_C{i}": torch.randint(0, r, (n,), generator=g, dtype=torch.int32)
            for i, r in enumerate(F_ROWS)}
    for i in range(N_DENSE):
        data[f"c_n_I{i}"] = torch.rand(n, generator=g)
    data["label"] = (torch.rand(n, generator=g) < 0.3).to(torch.int32)
    return data


def _reference_model():
    from pytorchrec_amd.model import DeepFM
    sparse, dense, label = _columns()
    torch.manual_seed(0)
    return DeepFM(sparse, dense, label, emb_size=DIM, layers=LAYERS, random_seed=7)


def _train(model, batches):
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    opt = torch.optim.SGD(model.get_parameters(), lr=LR)
    model.compile(opt, BCEWithLogitsLoss(), [], torch.device("cpu"))
    return [float(model.train_step(b)["loss"].detach()) for b in batches]


def _worker(rank, world, port, out_dir, steps, chunk_batch=None):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pytorchrec_amd.model import DeepFM
        from pytorchrec_amd.sharding import ShardComm, ShardedEmbeddingBank, sharded_tables
        if chunk_batch:  # the batch goes out as chunks (sub-senders) of this many samples
            ShardedEmbeddingBank.chunk_batch = chunk_batch
        comm = ShardComm()
        ref = _reference_model()  # same init on every rank: the global tables to shard
        sparse, dense, label = _columns()
        with sharded_tables(comm, cap=B):
            model = DeepFM(sparse, dense, label, emb_size=DIM, layers=LAYERS, random_seed=7)
        tables = [ref.embeddings.weight[o:o + n] for o, n in
                  zip(ref.embeddings.row_offset, ref.embeddings.category_nums)]
        model.embeddings.load_global_(tables)
        dense_sd = {k: v for k, v in ref.state_dict().items() if not k.startswith("embeddings")}
        model.load_state_dict(dense_sd, strict=False)
        model.distribute(comm)
        batches = []
        for s in range(steps):
            full = _batch(100 + s, B * world)
            batches.append({k: v[rank * B:(rank + 1) * B] for k, v in full.items()})
        losses = _train(model, batches)
        out = {"losses": np.array(losses)}
        for k, v in model.state_dict().items():
            out[k.replace(".", "__")] = v.detach().numpy()
        # sharded checkpoint: full bank in the unsharded layout on every rank, and a
        # fresh sharded replica restored from it holds exactly this rank's rows
        gsd = model.global_state_dict()
        out["global_bank"] = gsd["embeddings.weight"].detach().numpy()
        with sharded_tables(comm, cap=B):
            fresh = DeepFM(sparse, dense, label, emb_size=DIM, layers=LAYERS, random_seed=99)
        fresh.load_global_state_dict(gsd)
        cols = model.embeddings.dim + 1
        same = torch.equal(fresh.embeddings.weight[:, :cols], model.embeddings.weight[:, :cols])
        for k, v in model.state_dict().items():
            if not k.startswith("embeddings"):
                same = same and torch.equal(fresh.state_dict()[k], v)
        out["reload_ok"] = np.array(bool(same))
        # the row-sharded checkpoint (checkpoint.py): collective save_weights writes
        # per-rank shard files + rank 0's index; a fresh replica reads its own file
        ck = os.path.join(out_dir, "ckpt.pt")
        model.save_weights(ck)
        with sharded_tables(comm, cap=B):
            fresh2 = DeepFM(sparse, dense, label, emb_size=DIM, layers=LAYERS, random_seed=123)
        fresh2.load_weights(ck, torch.device("cpu"))
        same2 = torch.equal(fresh2.embeddings.weight[:, :cols], model.embeddings.weight[:, :cols])
        for k, v in model.state_dict().items():
            if not k.startswith("embeddings"):
                same2 = same2 and torch.equal(fresh2.state_dict()[k], v)
        out["ckpt_reload_ok"] = np.array(bool(same2))
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("steps,chunk_batch", [(2, None), (2, 12)])
def test_two_rank_sharded_deepfm_matches_single_process(steps, chunk_batch):
    """``chunk_batch`` 12: each rank's 32-sample batch goes out as 3 chunks (the
    compact exchange's sub-senders, as a batch past 8192 samples does on the GPU):
    an id repeated across chunks is sent once per chunk and summed by its owner."""
    import torch.multiprocessing as mp
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, steps, chunk_batch), nprocs=world,
                 join=True)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
        # the world-2 checkpoint into ONE unsharded model: the global tables
        unsharded = _reference_model()
        unsharded.load_weights(os.path.join(d, "ckpt.pt"), torch.device("cpu"))
        ckpt_bank = unsharded.embeddings.weight.detach().numpy()
    ref = _reference_model()
    ref_losses = _train(ref, [_batch(100 + s, B * world) for s in range(steps)])
    # the global loss is the mean of the ranks' (equal-size) batch means
    got = (res[0]["losses"] + res[1]["losses"]) / 2
    np.testing.assert_allclose(got, ref_losses, rtol=1e-5, atol=1e-6)
    sd = ref.state_dict()
    for k, v in sd.items():
        if k.startswith("embeddings"):
            continue
        for r in range(world):
            np.testing.assert_allclose(res[r][k.replace(".", "__")], v.numpy(), rtol=1e-5,
                                       atol=1e-6, err_msg=k)
    bank = ref.embeddings
    cols = bank.dim + 1
    for r in range(world):
        assert bool(res[r]["reload_ok"]), f"rank {r}: load_global_state_dict did not restore"
        assert bool(res[r]["ckpt_reload_ok"]), f"rank {r}: load_weights did not restore"
        assert res[r]["global_bank"].shape == tuple(bank.weight.shape)
        np.testing.assert_allclose(res[r]["global_bank"][:, :cols],
                                   bank.weight.detach()[:, :cols].numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(ckpt_bank[:, :cols], res[0]["global_bank"][:, :cols])
    for r in range(world):
        w = res[r]["embeddings__weight"]
        o_local = 0
        for f, (o, n) in enumerate(zip(bank.row_offset, bank.category_nums)):
            rows = bank.weight.detach()[o:o + n][r::world, :cols].numpy()
            np.testing.assert_allclose(w[o_local:o_local + rows.shape[0], :cols], rows,
                                       rtol=1e-5, atol=1e-6, err_msg=f"rank {r} table {f}")
            o_local += rows.shape[0]


def _worker_replicated(rank, world, port, out_dir, steps):
    """Unsharded (replicated) tables under distribute(), compiled BEFORE distribute:
    the bank must leave the per-rank fused update and train through the all-reduce
    (ADVICE r01); a sharded bank with weight_decay must be refused."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pytorchrec_amd.loss import BCEWithLogitsLoss
        from pytorchrec_amd.model import DeepFM
        from pytorchrec_amd.sharding import ShardComm, sharded_tables
        comm = ShardComm()
        model = _reference_model()
        if rank == 1:  # a different local init: distribute() must broadcast rank 0's
            with torch.no_grad():
                model.embeddings.weight.mul_(3.0)
        opt = torch.optim.SGD(model.get_parameters(), lr=LR)
        model.compile(opt, BCEWithLogitsLoss(), [], torch.device("cpu"))
        assert model.embeddings.update == "sgd"
        model.distribute(comm)
        assert model.embeddings.update == "dense"
        losses = []
        for s in range(steps):
            full = _batch(100 + s, B * world)
            losses.append(float(model.train_step(
                {k: v[rank * B:(rank + 1) * B] for k, v in full.items()})["loss"].detach()))
        out = {"losses": np.array(losses)}
        for k, v in model.state_dict().items():
            out[k.replace(".", "__")] = v.detach().numpy()
        sparse, dense, label = _columns()
        with sharded_tables(comm, cap=B):
            sh = DeepFM(sparse, dense, label, emb_size=DIM, layers=LAYERS, random_seed=7)
        refused = False
        try:
            sh.compile(torch.optim.SGD(sh.get_parameters(), lr=LR, weight_decay=1e-4),
                       BCEWithLogitsLoss(), [], torch.device("cpu"))
        except NotImplementedError:
            refused = True
        out["wd_refused"] = np.array(refused)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


def test_two_rank_replicated_tables_stay_identical():
    import torch.multiprocessing as mp
    world, steps = 2, 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_replicated, args=(world, _free_port(), d, steps), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    ref = _reference_model()
    ref_losses = _train(ref, [_batch(100 + s, B * world) for s in range(steps)])
    np.testing.assert_allclose((res[0]["losses"] + res[1]["losses"]) / 2, ref_losses, rtol=1e-5,
                               atol=1e-6)
    for k, v in ref.state_dict().items():
        key = k.replace(".", "__")
        assert np.array_equal(res[0][key], res[1][key]), f"replicas diverged: {k}"
        np.testing.assert_allclose(res[0][key], v.numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
    assert bool(res[0]["wd_refused"]) and bool(res[1]["wd_refused"])


def test_cpu_bucketize_slots_are_stable_and_complete():
    from pytorchrec_amd.sharding import ShardComm, ShardedEmbeddingBank, cpu_bucketize
    comm = ShardComm(world=3, rank=1)
    bank = ShardedEmbeddingBank([10, 31], 4, comm, cap=8)
    ids = [torch.tensor([0, 3, 6, 1, 9, 4, 2], dtype=torch.int32),
           torch.tensor([30, 2, 2, 5, 29, 0, 11], dtype=torch.int32)]
    send, pos = cpu_bucketize(bank, ids)
    assert send.shape == (3, 2, 8) and pos.shape == (2, 7)
    flat = send.reshape(-1)
    for f, t in enumerate(ids):
        for b, i in enumerate(t.tolist()):
            p = int(pos[f, b])
            owner, rem = divmod(p, 2 * 8)
            assert owner == i % 3 and rem // 8 == f
            assert int(flat[p]) == i // 3
    # stable: owner 0 of table 0 gets ids 0, 3, 6, 9 in sample order
    assert send[0, 0, :4].tolist() == [0, 1, 2, 3] and send[0, 0, 4:].tolist() == [-1] * 4
    with pytest.raises(IndexError):
        cpu_bucketize(bank, [torch.tensor([10], dtype=torch.int32), torch.tensor([0], dtype=torch.int32)])
    small = ShardedEmbeddingBank([10, 31], 4, comm, cap=1)
    with pytest.raises(RuntimeError, match="overflow"):
        cpu_bucketize(small, [torch.tensor([0, 3], dtype=torch.int32), torch.tensor([1, 2], dtype=torch.int32)])


def test_shard_row_split():
    from pytorchrec_amd.sharding import ShardComm, ShardedEmbeddingBank
    rows = [10, 7, 1]
    got = [ShardedEmbeddingBank(rows, 4, ShardComm(world=3, rank=r)).category_nums for r in range(3)]
    assert got == [[4, 3, 1], [3, 2, 0], [3, 2, 0]]
    assert [sum(g[f] for g in got) for f in range(3)] == rows


def test_compact_exchange_wire_bytes_c5_w8():
    """Sizing at the C5 shape (W = 8, B = 4096, 26 tables of 100M rows, bf16 D = 16 +
    w): <= 4 MB per rank and direction in the compact exchange, on CPU (no device)."""
    from pytorchrec_amd import sharding as S
    W, B, F, R = 8, 4096, 26, 100_000_000
    cap = S.default_cap(B, W, [R] * F)
    cap_rows = S.default_cap_rows(B, W, [R] * F, cap)
    rec = 36  # mrec_shard_wire_bytes(16, 1, bf16)
    remote = (W - 1) * cap_rows * rec  # the part for this rank stays local
    assert cap_rows * W * rec <= 4.1e6 and remote <= 4e6, (cap_rows, remote)


def test_cpu_bucketize_dedup_layout():
    """The compact ids message on the CPU: per (owner, table) the distinct ids in
    quarter-major, then first-lookup order (as local ids; ABI 28: the GPU bucketize
    runs one workgroup per quarter of the ids, sharding.dedup_quarter), -1 padding,
    the counts header, and every lookup's pos pointing at its id's slot."""
    from pytorchrec_amd.sharding import (ShardComm, ShardedEmbeddingBank, cpu_bucketize_dedup,
                                         dedup_quarter)
    W, B = 3, 40
    rows = [17, 5, 1000]
    bank = ShardedEmbeddingBank(rows, 8, ShardComm(world=W, rank=0), cap=B, max_batch=B)
    g = torch.Generator().manual_seed(0)
    ids = [torch.randint(0, n, (B,), generator=g, dtype=torch.int32) for n in rows]
    send, pos = cpu_bucketize_dedup(bank, ids)
    F, cap = len(rows), bank.cap
    for f, t in enumerate(ids):
        for o in range(W):
            seen = []
            for b in range(B):
                i = int(t[b])
                if i % W == o and i not in seen:
                    seen.append(i)
            q = dedup_quarter(torch.tensor(seen, dtype=torch.long), bank.dedup_quarters).tolist()
            seen = [i for _, _, i in sorted((qq, k, i) for k, (qq, i) in enumerate(zip(q, seen)))]
            cnt = int(send[o, F * cap + f])
            assert cnt == len(seen)
            assert send[o, f * cap:f * cap + cnt].tolist() == [i // W for i in seen]
            assert bool((send[o, f * cap + cnt:(f + 1) * cap] == -1).all())
        for b in range(B):
            i = int(t[b])
            p = int(pos[f, b])
            o, rest = divmod(p, F * cap)
            assert o == i % W and rest // cap == f
            assert int(send[o, f * cap + rest % cap]) == i // W
