"""Row-sharded checkpoints (pytorchrec_amd/checkpoint.py; SURVEY.md §8(f) rank 4,
reference IModel.save_weights / load_weights IModel.py:73-81 and
ModelCheckpoint._save_model ModelCheckpoint.py:66-91), on the CPU.

W ranks' shards are written from ONE process through a communicator whose
collectives are no-ops (the file format does not depend on them); every load is
checked row by row against the global tables:

  * same world size: each rank reads only its own shard file;
  * resharding to W' in {1 (an unsharded EmbeddingBank), 2, 3, 5}: every rank holds
    exactly global rows r', r' + W', ... of every table, bitwise (fp32 and bf16);
  * a plain single-file state dict of the unsharded model loads into a sharded one;
  * save_best_weights right after save_weights keeps hard links (no copy), which a
    later save to the same path does not change.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

ROWS = [50, 7, 129, 1, 1000]
DIM = 8


class _LocalComm:
    """A ShardComm stand-in for (world, rank) with no-op collectives -- except that
    the ranks of one simulated save (saved one after another, rank 0 first) share
    rank 0's contribution to a 3-element all-reduce, as the save id's sum would."""

    _rank0_sum = None

    def __init__(self, world, rank):
        self.world, self.rank, self.group, self.force = world, rank, None, False

    def allreduce_sum_(self, t):
        if t.numel() == 3:
            if self.rank == 0:
                _LocalComm._rank0_sum = t.clone()
            else:
                t.copy_(_LocalComm._rank0_sum)
        return t


def _model(world=None, rank=0, dtype=torch.float32, seed=7):
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    from pytorchrec_amd.sharding import sharded_tables
    sparse = [CategoricalColumnWithIdentity(n, f"c_c_C{i}") for i, n in enumerate(ROWS)]
    dense = [NumericColumn(f"c_n_I{i}") for i in range(3)]
    label = CategoricalColumnWithIdentity(2, "label")
    mk = lambda: DeepFM(sparse, dense, label, emb_size=DIM, layers=(16, 8), emb_dtype=dtype,  # noqa: E731
                        random_seed=seed)
    if world is None:
        return mk()
    with sharded_tables(_LocalComm(world, rank)):
        return mk()


def _global_tables(dtype):
    g = torch.Generator().manual_seed(11)
    return [torch.randn(n, DIM + 1, generator=g).to(dtype) for n in ROWS]


def _save_world(path, world, dtype, tables):
    from pytorchrec_amd import checkpoint
    ms = []
    for r in range(world):
        m = _model(world, r, dtype)
        m.embeddings.load_global_(tables)
        checkpoint.save_sharded(m, path)
        ms.append(m)
    return ms


def _check_rows(m, tables, world, rank):
    cols = DIM + 1
    for f, t in enumerate(tables):
        o, n = m.embeddings.row_offset[f], m.embeddings.category_nums[f]
        got = m.embeddings.weight[o:o + n, :cols]
        want = t[rank::world, :cols]
        assert torch.equal(got.view(torch.int16) if got.dtype == torch.bfloat16 else got,
                           want.view(torch.int16) if want.dtype == torch.bfloat16 else want), \
            (world, rank, f)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_sharded_checkpoint_reshards_bitwise(dtype):
    from pytorchrec_amd import checkpoint
    tables = _global_tables(dtype)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ckpt.pt")
        src = _save_world(path, 4, dtype, tables)
        files = sorted(os.listdir(d))
        assert files == sorted(["ckpt.pt"] + [f"ckpt.pt.embeddings.weight.r{r}of4.npy{x}"
                                              for r in range(4) for x in ("", ".id")]), files
        state = torch.load(path, map_location="cpu", weights_only=True)
        assert "embeddings.weight" not in state and checkpoint.INDEX_KEY in state
        # the dense entries are saved under their unsharded keys
        for k, v in src[0].state_dict().items():
            if k != "embeddings.weight":
                assert torch.equal(state[k], v), k
        for world in (4, 2, 3, 5):
            for r in range(world):
                m = _model(world, r, dtype, seed=99)
                if world == 4:  # same world size: only the rank's own file is read
                    for q in range(4):
                        if q != r:
                            os.rename(checkpoint.shard_file(path, "embeddings.weight", q, 4),
                                      os.path.join(d, f"hidden{q}"))
                checkpoint.load_into(m, state, path)
                if world == 4:
                    for q in range(4):
                        if q != r:
                            os.rename(os.path.join(d, f"hidden{q}"),
                                      checkpoint.shard_file(path, "embeddings.weight", q, 4))
                _check_rows(m, tables, world, r)
                for k, v in src[0].state_dict().items():
                    if k != "embeddings.weight":
                        assert torch.equal(m.state_dict()[k], v), k
        u = _model(None, 0, dtype, seed=99)  # unsharded EmbeddingBank: world 1
        checkpoint.load_into(u, state, path)
        _check_rows(u, tables, 1, 0)
        # a model of a different table count / dim is refused
        bad = _model(None, 0, dtype)
        bad.embeddings.dim = DIM + 1
        with pytest.raises(ValueError):
            checkpoint.load_into(bad, state, path)


def test_unsharded_state_dict_loads_into_sharded_and_best_weights_link():
    from pytorchrec_amd import checkpoint
    tables = _global_tables(torch.float32)
    u = _model(None)
    with torch.no_grad():
        for f, t in enumerate(tables):
            o, n = u.embeddings.row_offset[f], u.embeddings.category_nums[f]
            u.embeddings.weight[o:o + n, :DIM + 1] = t
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "single.pt")
        u.save_weights(path)  # the reference's format: one state dict
        for r in range(3):
            m = _model(3, r, seed=99)
            m.load_weights(path, torch.device("cpu"))
            _check_rows(m, tables, 3, r)
        # save_best_weights of an unsharded model: the reference's host copy
        # (IModel.py:314-315), no file
        u.save_best_weights()
        assert not os.path.exists(path + ".best")
        with torch.no_grad():
            u.embeddings.weight.add_(1.0)
        u._weights_version += 1
        u.save_weights(path)
        u.compiled_device = torch.device("cpu")
        u.load_best_weights()
        _check_rows(u, tables, 1, 0)
        # sharded: every rank links its own shard files
        ms = _save_world(os.path.join(d, "sh.pt"), 2, torch.float32, tables)
        for m in ms:
            m._last_saved = (os.path.join(d, "sh.pt"), m._weights_version)
            m.save_best_weights()
        for r in range(2):
            assert os.path.samefile(os.path.join(d, f"sh.pt.best.embeddings.weight.r{r}of2.npy"),
                                    os.path.join(d, f"sh.pt.embeddings.weight.r{r}of2.npy"))
        assert os.path.samefile(os.path.join(d, "sh.pt.best"), os.path.join(d, "sh.pt"))
        m = _model(2, 1, seed=5)
        m.load_weights(os.path.join(d, "sh.pt.best"), torch.device("cpu"))
        _check_rows(m, tables, 2, 1)
        checkpoint.remove_checkpoint(os.path.join(d, "sh.pt"))
        assert not any(n.startswith("sh.pt.embeddings") for n in os.listdir(d))
        assert np.all([os.path.exists(os.path.join(d, f"sh.pt.best.embeddings.weight.r{r}of2.npy"))
                       for r in range(2)])


def test_sharded_checkpoint_with_a_shard_of_another_save_is_refused():
    """a crash between the shards' renames and the index leaves a new
    index beside shard files of the previous save (same shapes).  The save id in the
    index and beside every shard makes the load raise instead of mixing two steps."""
    import shutil
    from pytorchrec_amd import checkpoint
    tables = _global_tables(torch.float32)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "c.pt")
        _save_world(path, 2, torch.float32, tables)
        old = checkpoint.shard_file(path, "embeddings.weight", 1, 2)
        shutil.copy(old, old + ".prev")
        shutil.copy(checkpoint.id_file(old), old + ".prev.id")
        newer = [t + 1 for t in tables]
        _save_world(path, 2, torch.float32, newer)
        state = torch.load(path, map_location="cpu", weights_only=True)
        ids = {meta["save_id"] for meta in state[checkpoint.INDEX_KEY].values()}
        assert len(ids) == 1
        m = _model(2, 1, seed=5)
        checkpoint.load_into(m, state, path)
        _check_rows(m, newer, 2, 1)
        os.replace(old + ".prev", old)  # rank 1 "crashed" before its rename
        os.replace(old + ".prev.id", checkpoint.id_file(old))
        with pytest.raises(RuntimeError, match="another save"):
            checkpoint.load_into(_model(2, 1, seed=5), state, path)
        os.remove(checkpoint.id_file(old))  # or before it wrote its id
        with pytest.raises(RuntimeError, match="another save"):
            checkpoint.load_into(_model(2, 1, seed=5), state, path)
