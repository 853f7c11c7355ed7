"""The N > 1 row-sharded DeepFM step as REAL processes on the GPU.

Two ranks, each its own process on cuda:0 (the one-GPU box), exchanging over
``gloo`` with CUDA tensors (gloo stages them through host memory: a rehearsal of
the process-level protocol, not a bandwidth measurement; RCCL refuses two ranks
on one device).  Every kernel of the N > 1 path runs: compact exchange (distinct
ids per (owner, table), 36-B records both ways), the sender's and owner's
backward plans, the owner's fused SGD with lr / W, the dense all-reduce.

Checked against ONE process training the unsharded model on the concatenation of
both ranks' batches (fp32 tables, so only the summation order of a row's gradient
differs -- per rank first, then rank order -- and of the dense weight gradients):
losses, dense parameters and every shard's rows within 1e-5 relative.  A second
case runs bf16 tables at the C2 shape's width (26 tables, 400-wide tower) and
checks the loss trajectory and the shard rows to bf16 tolerance.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LR = 0.05


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spec(case):
    if case == "small_fp32":
        return dict(rows=[5000, 7, 129, 1, 70000, 300], dim=16, n_dense=13, B=512,
                    layers=(64, 32), dtype=torch.float32, steps=3, opt="sgd")
    if case == "adam_bf16":  # lazy (dense-compatible) Adam on the compact exchange, bf16 rows
        return dict(rows=[5000, 7, 129, 1, 70000, 300], dim=16, n_dense=13, B=512,
                    layers=(64, 32), dtype=torch.bfloat16, steps=3, opt="adam")
    return dict(rows=[38462] * 26, dim=16, n_dense=13, B=1024, layers=(400, 400, 400),
                dtype=torch.bfloat16, steps=3, opt="sgd")


def _columns(sp):
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{i}") for i, n in enumerate(sp["rows"])]
    dense = [NumericColumn(f"c_n_I{i}") for i in range(sp["n_dense"])]
    label = CategoricalColumnWithIdentity(2, "label")
    return sparse, dense, label


def _batch(sp, seed, n, dev):
    g = torch.Generator().manual_seed(seed)
    data = {f"c_c_C{i}": torch.randint(0, r, (n,), generator=g, dtype=torch.int32)
            for i, r in enumerate(sp["rows"])}
    for i in range(sp["n_dense"]):
        data[f"c_n_I{i}"] = torch.rand(n, generator=g)
    data["label"] = (torch.rand(n, generator=g) < 0.3).to(torch.float32)
    return {k: v.to(dev) for k, v in data.items()}


def _model(sp, dev):
    from pytorchrec_amd.model import DeepFM
    sparse, dense, label = _columns(sp)
    m = DeepFM(sparse, dense, label, emb_size=sp["dim"], layers=sp["layers"], dropout=0.0,
               emb_dtype=sp["dtype"], device=dev, random_seed=7)
    for b in m.embedding_banks():
        b.stochastic_rounding = False
    return m


def _train(model, batches, dev, opt="sgd"):
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    o = (torch.optim.SGD(model.get_parameters(), lr=LR) if opt == "sgd" else
         torch.optim.Adam(model.get_parameters(), lr=1e-3))
    model.compile(o, BCEWithLogitsLoss(), [], dev)
    return [float(model.train_step(b)["loss"].detach()) for b in batches]


def _worker(rank, world, port, out_dir, case):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pytorchrec_amd.model import DeepFM
        from pytorchrec_amd.sharding import ShardComm, sharded_tables
        sp = _spec(case)
        comm = ShardComm()
        ref = _model(sp, dev)  # same init on every rank: the global tables to shard
        sparse, dense, label = _columns(sp)
        with sharded_tables(comm, max_batch=sp["B"]):
            model = DeepFM(sparse, dense, label, emb_size=sp["dim"], layers=sp["layers"],
                           dropout=0.0, emb_dtype=sp["dtype"], device=dev, random_seed=7)
        tables = [ref.embeddings.weight[o:o + n] for o, n in
                  zip(ref.embeddings.row_offset, ref.embeddings.category_nums)]
        model.embeddings.load_global_(tables)
        model.embeddings.stochastic_rounding = False
        dense_sd = {k: v for k, v in ref.state_dict().items() if not k.startswith("embeddings")}
        model.load_state_dict(dense_sd, strict=False)
        model.distribute(comm)
        assert model.embeddings.use_compact(sp["B"]), "N > 1 must take the compact exchange"
        batches = []
        for s in range(sp["steps"]):
            full = _batch(sp, 100 + s, sp["B"] * world, dev)
            batches.append({k: v[rank * sp["B"]:(rank + 1) * sp["B"]] for k, v in full.items()})
        losses = _train(model, batches, dev, sp["opt"])
        if sp["opt"] == "adam":
            assert model.embeddings.update == "adam", model.embeddings.update
        torch.cuda.synchronize()
        out = {"losses": np.array(losses)}
        for k, v in model.state_dict().items():
            out[k.replace(".", "__")] = v.detach().float().cpu().numpy()
        # the row-sharded checkpoint (checkpoint.py): every rank writes its shard, a
        # fresh sharded replica reads its own file back bit-identically
        ck = os.path.join(out_dir, "ckpt.pt")
        model.save_weights(ck)
        with sharded_tables(comm, max_batch=sp["B"]):
            fresh = DeepFM(sparse, dense, label, emb_size=sp["dim"], layers=sp["layers"],
                           dropout=0.0, emb_dtype=sp["dtype"], device=dev, random_seed=99)
        fresh.load_weights(ck, dev)
        same = torch.equal(fresh.embeddings.weight, model.embeddings.weight)
        for k, v in model.state_dict().items():
            same = same and torch.equal(fresh.state_dict()[k], v)
        out["ckpt_reload_ok"] = np.array(bool(same))
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["small_fp32", "c2_width_bf16", "adam_bf16"])
def test_two_process_sharded_step_on_gpu_matches_single_process(gpu, case):
    import torch.multiprocessing as mp
    world = 2
    sp = _spec(case)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, case), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
        # the world-2 checkpoint resharded into ONE unsharded model on the GPU: global
        # row i = local row i // 2 of rank i % 2, bit for bit
        u = _model(sp, gpu)
        u.load_weights(os.path.join(d, "ckpt.pt"), gpu)
        ubank = u.embeddings.weight.detach().float().cpu().numpy()
        for r in range(world):
            assert bool(res[r]["ckpt_reload_ok"]), f"rank {r}: load_weights did not restore"
            o_local = 0
            for o, n in zip(u.embeddings.row_offset, u.embeddings.category_nums):
                k = len(range(r, n, world))
                np.testing.assert_array_equal(
                    ubank[o:o + n][r::world, :sp["dim"] + 1],
                    res[r]["embeddings__weight"][o_local:o_local + k, :sp["dim"] + 1])
                o_local += k
        del u
    ref = _model(sp, gpu)
    ref_losses = _train(ref, [_batch(sp, 100 + s, sp["B"] * world, gpu)
                              for s in range(sp["steps"])], gpu, sp["opt"])
    fp32 = sp["dtype"] == torch.float32
    # the global loss is the mean of the ranks' (equal-size) batch means
    got = (res[0]["losses"] + res[1]["losses"]) / 2
    np.testing.assert_allclose(got, ref_losses, rtol=1e-5 if fp32 else 2e-3, atol=1e-6)
    rtol, atol = (1e-5, 1e-6) if fp32 else (2e-2, 2e-3)
    sd = ref.state_dict()
    for k, v in sd.items():
        if k.startswith("embeddings"):
            continue
        for r in range(world):
            np.testing.assert_allclose(res[r][k.replace(".", "__")], v.detach().float().cpu().numpy(),
                                       rtol=rtol, atol=atol, err_msg=k)
    bank = ref.embeddings
    cols = bank.dim + 1
    W = bank.weight.detach().float().cpu()
    for r in range(world):
        w = res[r]["embeddings__weight"]
        o_local = 0
        for f, (o, n) in enumerate(zip(bank.row_offset, bank.category_nums)):
            rows = W[o:o + n][r::world, :cols].numpy()
            got_rows = w[o_local:o_local + rows.shape[0], :cols]
            if fp32:
                np.testing.assert_allclose(got_rows, rows, rtol=1e-5, atol=1e-7,
                                           err_msg=f"rank {r} table {f}")
            elif sp["opt"] == "sgd":  # bf16 rows: one bf16 ulp (2^-8 relative) apart, few differ
                diff = np.abs(got_rows - rows)
                assert np.all(diff <= 2.0 ** -7 * np.abs(rows) + 1e-6), f"rank {r} table {f}"
                assert np.mean(diff > 0) < 0.01, f"rank {r} table {f}: {np.mean(diff > 0)}"
            else:  # lazy Adam, bf16: each rank's row-gradient sum crosses the wire rounded
                # to bf16 once (and is summed per rank first).  Adam's step is normalised:
                # where a gradient element is tiny against that rounding its sign can flip,
                # moving the element by up to 2 lr per step -- so: every element within
                # 2 lr x steps (+ 2^-6 relative), and at most 2 % beyond one bf16 ulp
                diff = np.abs(got_rows - rows)
                lim = 2 * 1e-3 * sp["steps"] + 2.0 ** -6 * np.abs(rows)
                far = float(np.mean(diff > 2.0 ** -7 * np.abs(rows) + 1e-6)) if diff.size else 0.0
                assert np.all(diff <= lim), (r, f, float((diff / lim).max()), far)
                assert far < 0.02, (r, f, far, float(np.mean(diff > 0)))
            o_local += rows.shape[0]
