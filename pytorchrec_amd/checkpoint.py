"""Row-sharded checkpoints.

The reference saves and restores a model as one pickled ``state_dict``
(``IModel.save_weights`` / ``load_weights``, torchrec/model/IModel.py:73-81, driven
by ``ModelCheckpoint._save_model``, torchrec/callback/ModelCheckpoint.py:66-91).
For a row-sharded bank (config C5: 26 x 10^8 rows, 166 GB, ~21 GB per GPU at W = 8)
that single tensor cannot be assembled anywhere, so a sharded model writes:

  * ``filepath`` (rank 0, ``torch.save``, loadable with ``weights_only=True``): every
    non-bank entry of the state dict under its usual key, plus ``INDEX_KEY`` ->
    {bank key: {"world", "global_rows", "row_stride", "dim", "has_w", "dtype",
    "files"}} describing the bank ("files": the shard files' names relative to the
    main file's own name, so a renamed or linked checkpoint stays whole);
  * ``{filepath}.{bank key}.r{r}of{W}.npy`` (every rank, its own shard): the local
    rows [local_rows, row_stride] in the bank's dtype (bf16 stored as its uint16
    bits), written by device -> host chunks of ``chunk_rows`` rows -- no rank holds
    more than one chunk of it in host memory, and no GPU holds more than its shard.

Every file is written under a temporary name and renamed into place, so a new save
never modifies the inode of an earlier one (``link_snapshot`` relies on it).

Crash consistency: a save draws one random ``save_id`` (rank 0's, shared by an
all-reduce), written into the index and beside every shard file (``{shard}.id``);
rank 0 writes the main file only after a barrier that follows every rank's renames.
Loading checks each shard's id against the index, so a crash mid-save (new index,
some shards of the previous save: same shapes) raises instead of restoring rows of
two different steps.  The main file is read by every rank (``load_weights``), so
it must live on a filesystem all ranks see; at the same world size each rank then
reads only its own shard files (those may be node-local).

Loading reads only the rows the loading rank owns, straight from the shard files
(numpy memory maps, ``allow_pickle=False``): same world size -> its own file, chunk
by chunk; any other world size (including an unsharded ``EmbeddingBank``, world 1)
-> for every source shard s the rows g = s + j W (j local) with g % W' == r', in
chunks.  A single-file checkpoint of the unsharded model (a plain ``state_dict``)
still loads into a sharded model, and a sharded checkpoint into an unsharded one.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

INDEX_KEY = "__mrec_sharded_banks__"
CHUNK_ROWS = 1 << 22  # rows per device <-> host chunk (256 MB of 64-B rows)


def _banks(model) -> List[Tuple[str, torch.nn.Module]]:
    from pytorchrec_amd.embedding import EmbeddingBank
    return [((name + "." if name else "") + "weight", m) for name, m in model.named_modules()
            if isinstance(m, EmbeddingBank)]


def _is_sharded(m) -> bool:
    from pytorchrec_amd.sharding import ShardedEmbeddingBank
    return isinstance(m, ShardedEmbeddingBank)


def _shard_layout(global_rows: List[int], world: int, rank: int) -> Tuple[List[int], List[int]]:
    """(local rows per table, local row offset per table) of shard ``rank`` of
    ``world`` (ShardedEmbeddingBank: local table f = global rows rank, rank + W, ...)."""
    n = [(g - rank + world - 1) // world if g > rank else 0 for g in global_rows]
    offs, acc = [], 0
    for v in n:
        offs.append(acc)
        acc += v
    return n, offs


def shard_suffix(key: str, rank: int, world: int) -> str:
    return f".{key}.r{rank}of{world}.npy"


def shard_file(filepath: str, key: str, rank: int, world: int) -> str:
    return filepath + shard_suffix(key, rank, world)


def _np_view(t: torch.Tensor) -> np.ndarray:
    """A host tensor's bytes as numpy (bf16 -> its uint16 bits)."""
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _torch_view(a: np.ndarray, dtype: str) -> torch.Tensor:
    t = torch.from_numpy(np.array(a, copy=True))  # (out of the read-only memory map)
    if dtype == "bfloat16":
        return t.view(torch.int16).view(torch.bfloat16)
    return t


def _barrier(comm, device):
    comm.allreduce_sum_(torch.zeros(1, device=device))


def _shared_save_id(comm, rank: int, device) -> int:
    """A random 48-bit id drawn by rank 0 and summed to every rank (three 16-bit
    parts: exact in fp32, whatever the communicator reduces in)."""
    parts = torch.zeros(3, device=device)
    if rank == 0:
        parts.copy_(torch.from_numpy(np.frombuffer(os.urandom(6), dtype=np.uint16)
                                     .astype(np.float32)))
    comm.allreduce_sum_(parts)
    a, b, c = (int(v) for v in parts.cpu().tolist())
    return (a << 32) | (b << 16) | c


def id_file(shard_path: str) -> str:
    return shard_path + ".id"


def _write_text(path: str, text: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


@torch.no_grad()
def save_sharded(model, filepath: str, chunk_rows: int = CHUNK_ROWS) -> None:
    """Write ``model`` (with row-sharded banks) as described in the module
    docstring.  Collective: every rank of the banks' communicator calls it."""
    sd = model.state_dict()  # (brings lazily-updated rows current first)
    banks = _banks(model)
    sharded = [(k, m) for k, m in banks if _is_sharded(m)]
    comm = sharded[0][1].comm
    rank, world = sharded[0][1].rank, sharded[0][1].world
    dev = sharded[0][1].weight.device
    save_id = _shared_save_id(comm, rank, dev)
    index = {}
    for key, m in sharded:
        dt = "bfloat16" if m.weight.dtype == torch.bfloat16 else "float32"
        path = shard_file(filepath, key, m.rank, m.world)
        tmp = path + ".tmp.npy"
        arr = np.lib.format.open_memmap(tmp, mode="w+", dtype=np.uint16 if dt == "bfloat16"
                                        else np.float32, shape=(m.total_rows, m.row_stride))
        for a in range(0, m.total_rows, chunk_rows):
            b = min(m.total_rows, a + chunk_rows)
            arr[a:b] = _np_view(m.weight[a:b].detach().cpu())
        arr.flush()
        del arr
        os.replace(tmp, path)
        _write_text(id_file(path), f"{save_id}\n")
        index[key] = {"world": m.world, "global_rows": list(m.global_rows),
                      "row_stride": m.row_stride, "dim": m.dim, "has_w": bool(m.has_w),
                      "dtype": dt, "files": [shard_suffix(key, r, m.world) for r in range(m.world)],
                      "save_id": save_id}
    _barrier(comm, dev)  # every rank's shards and ids are in place before the index
    if rank == 0:
        keys = {k for k, _ in sharded}
        out = {k: v for k, v in sd.items() if k not in keys}
        out[INDEX_KEY] = index
        save_file(out, filepath)
    _barrier(comm, dev)


def save_file(obj, filepath: str) -> None:
    """``torch.save`` under a temporary name, then renamed into place."""
    tmp = filepath + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, filepath)


def _target(m) -> Tuple[int, int, List[int]]:
    if _is_sharded(m):
        return m.world, m.rank, list(m.global_rows)
    return 1, 0, list(m.category_nums)


@torch.no_grad()
def load_bank_from_shards(m, meta: Dict, filepath: str, chunk_rows: int = CHUNK_ROWS) -> None:
    """Fill bank ``m`` (sharded at any world size, or unsharded) with its rows from
    the shard files ``meta`` describes.  Only the useful columns [dim (+ w)] are
    copied (the row pitch may differ with the dtype); the pad columns stay zero."""
    W, grows = int(meta["world"]), [int(g) for g in meta["global_rows"]]
    Wt, rt, tgrows = _target(m)
    if tgrows != grows:
        raise ValueError(f"checkpoint tables have {grows} rows, the bank {tgrows}")
    if int(meta["dim"]) != m.dim or bool(meta["has_w"]) != bool(m.has_w):
        raise ValueError("checkpoint bank dim / first-order column differ from the model's")
    cols = m.dim + (1 if m.has_w else 0)
    dev = m.weight.device
    _, toffs = _shard_layout(grows, Wt, rt)
    for s in range(W):
        if Wt == W and rt != s:
            continue  # same world size: only this rank's own file has its rows (and only
            # it needs to be visible to this rank: node-local disks work)
        path = filepath + meta["files"][s]
        if "save_id" in meta:  # (checkpoints before r06 carry none)
            try:
                with open(id_file(path)) as f:
                    got = int(f.read().strip())
            except (OSError, ValueError):
                got = None
            if got != int(meta["save_id"]):
                raise RuntimeError(f"{path}: shard of another save (id {got}, the index says "
                                   f"{meta['save_id']}): the checkpoint is incomplete")
        mm = np.load(path, mmap_mode="r", allow_pickle=False)
        n_s, offs_s = _shard_layout(grows, W, s)
        if mm.shape[0] != sum(n_s) or mm.shape[1] != int(meta["row_stride"]):
            raise ValueError(f"{path}: shape {mm.shape} does not match the index")
        for f, g_n in enumerate(grows):
            n = n_s[f]
            if n == 0:
                continue
            if Wt == W:  # contiguous: local row j -> local row j
                for a in range(0, n, chunk_rows):
                    b = min(n, a + chunk_rows)
                    src = _torch_view(mm[offs_s[f] + a:offs_s[f] + b, :cols], meta["dtype"])
                    m.weight[toffs[f] + a:toffs[f] + b, :cols] = src.to(dev, m.weight.dtype)
                continue
            # resharding: g = s + j W owned by rank g % Wt at local g // Wt; j runs over
            # an arithmetic progression of step Wt / gcd(W, Wt) (possibly empty)
            step = Wt // math.gcd(W, Wt)
            j0 = next((j for j in range(step) if (s + j * W) % Wt == rt), None)
            if j0 is None or j0 >= n:
                continue
            for a in range(j0, n, chunk_rows * step):
                js = np.arange(a, min(n, a + chunk_rows * step), step, dtype=np.int64)
                src = _torch_view(mm[offs_s[f] + js, :cols], meta["dtype"])
                dst = torch.from_numpy(toffs[f] + (s + js * W) // Wt).to(dev)
                m.weight[:, :cols].index_copy_(0, dst, src.to(dev, m.weight.dtype))
        del mm


@torch.no_grad()
def load_into(model, state: Dict, filepath: Optional[str] = None, strict: bool = True) -> None:
    """Load a checkpoint ``state`` (the main file ``filepath`` of a sharded
    checkpoint, or any single-file ``state_dict`` in the unsharded layout) into
    ``model``, sharded or not: every bank takes only its own rows."""
    sd = dict(state)
    index = sd.pop(INDEX_KEY, {})
    if not index and not has_sharded_banks(model):  # the reference's path (and key mapping)
        model.load_state_dict(sd, strict=strict)
        return
    bank_keys, missing = set(), []
    for key, m in _banks(model):
        if key in index or key in sd or _is_sharded(m):
            bank_keys.add(key)
        if key in index:
            if filepath is None:
                raise ValueError("a row-sharded checkpoint's state needs its file path")
            sd.pop(key, None)
            load_bank_from_shards(m, index[key], filepath)
        elif key in sd:
            full = sd.pop(key)
            if _is_sharded(m):
                m.load_global_bank_(full)
            else:
                if tuple(full.shape) != tuple(m.weight.shape):
                    raise ValueError(f"{key}: checkpoint shape {tuple(full.shape)} != "
                                     f"{tuple(m.weight.shape)}")
                m.weight.copy_(full.to(m.weight.device, m.weight.dtype))
        elif _is_sharded(m):
            missing.append(key)
    res = model.load_state_dict(sd, strict=False)
    missing += [k for k in res.missing_keys if k not in bank_keys]
    unexpected = list(res.unexpected_keys)
    if strict and (missing or unexpected):
        raise RuntimeError(f"Error(s) in loading state_dict for {type(model).__name__}: "
                           f"missing keys {missing}, unexpected keys {unexpected}")


def has_sharded_banks(model) -> bool:
    return any(_is_sharded(m) for _, m in _banks(model))


def checkpoint_files(model, filepath: str) -> List[str]:
    """The files of ``filepath`` this rank wrote: its shard files (+ the main file on
    rank 0, or the single file of an unsharded model)."""
    sharded = [(k, m) for k, m in _banks(model) if _is_sharded(m)]
    if not sharded:
        return [filepath]
    r, W = sharded[0][1].rank, sharded[0][1].world
    shards = [shard_file(filepath, k, r, W) for k, _ in sharded]
    return ([filepath] if r == 0 else []) + shards + [id_file(p) for p in shards]


def link_snapshot(model, filepath: str, snapshot: str) -> None:
    """Hard-link this rank's files of checkpoint ``filepath`` under the name
    ``snapshot`` (no copy; later saves to ``filepath`` replace its files with new
    inodes, so the snapshot keeps these bytes).  Every rank calls it."""
    for src in checkpoint_files(model, filepath):
        dst = snapshot + src[len(filepath):]
        if os.path.exists(dst):
            os.remove(dst)
        os.link(src, dst)


def remove_checkpoint(filepath: str, state: Optional[Dict] = None) -> None:
    """Delete a checkpoint's main file and the shard files its index names."""
    if state is None:
        state = torch.load(filepath, map_location="cpu", weights_only=True)
    for meta in state.get(INDEX_KEY, {}).values():
        for suf in meta["files"]:
            for p in (filepath + suf, id_file(filepath + suf)):
                if os.path.exists(p):
                    os.remove(p)
    if os.path.exists(filepath):
        os.remove(filepath)
