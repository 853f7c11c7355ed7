"""Row-sharded embedding tables across the GPUs of a node.

One process per GPU.  Table f is split cyclically: global id ``i`` lives on rank
``i % W`` as local row ``i // W`` (cyclic, so Zipf-hot rows spread over owners).
The dense tower stays data-parallel.  One training step of a sharded bank (the
compact exchange, include/mrec.h ABI 19):

  sender  distinct ids per (owner, table) into fixed-capacity    mrec_shard_bucketize_dedup
          slots, every lookup's slot (pos), per-table counts
          all_to_all ids                                         (equal split, RCCL)
  owner   rows of the received ids -> one 36-B record per        mrec_shard_gather_wire
          distinct row, packed per owner over all tables
          all_to_all records back                                (equal split)
  sender  records -> slot rows, the part prefixes of its own     mrec_shard_wire_unpack_ex
          record layout
          interaction on the slot rows, with the sender's        mrec_interact_fwd_ex
          backward plan over pos in the same launch
  ---- backward ----
  sender  gradient sum of each slot's lookups (fixed ascending   mrec_emb_bwd_apply_rec
          order) written straight as one record per distinct     (ABI 26; batches past
          row, table dtype                                       4096: DENSE_GRAD sums
                                                                 + mrec_shard_wire_pack)
          all_to_all records to the owners                       (equal split)
  owner   plan over the received ids (in the gather launch);     mrec_emb_bwd_apply_wire
          fixed-order sums over the senders read from the
          records in place + fused SGD

so the bytes on xGMI per rank and direction are ~cap_rows x 36 B per peer (one
record per distinct id; bf16, D = 16 + w) instead of n_tables x cap x 64 B rows
and 80-B fp32 gradients.  Banks under a fused lazy Adam take the same path: the
owner's wire gather catches each row up to the current step as it packs it
(ABI 25).  ``compact = False`` keeps the slot exchange of ABI 14 (one 64-B row /
fp32 gradient per lookup).  An owner whose exchange view (W * cap entries per
table) exceeds one plan workgroup sums the received gradients with the large-batch
bucketed plan (owner_apply_large).

Every exchange buffer has W equal parts, so all collectives are equal-split: no
host sync, capturable in a HIP graph.  An overflow (more distinct ids of one table
for one owner than ``cap``, or of all tables than ``cap_rows``) is flagged on the
device and raised, never dropped silently.  The loss is the mean over each rank's
batch, so the global objective is the mean of the ranks' losses: dense gradients
are all-reduced and averaged, and owners scale the summed row gradients by 1/W.
A row's gradient is summed per rank first (ascending sample order), then over the
ranks in rank order -- the data-parallel reduction order.

The reference has no sharding (it keeps one dense ``nn.Embedding`` per field,
FunkSVD.py:39-41); the per-field semantics (gather, duplicate-summing backward,
SGD) are unchanged.  The same protocol runs on CPU tensors over ``gloo`` (the
multi-process tests), with torch ops in place of the kernels.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from pytorchrec_amd import _mrec
from pytorchrec_amd.embedding import EmbeddingBank, _dense_first_order_grads, _trigger


# ----------------------------------------------------------------------------
# communicator
# ----------------------------------------------------------------------------


class ShardComm:
    """Equal-split all-to-all and mean all-reduce on a ``torch.distributed`` group
    (RCCL for GPU tensors, gloo for CPU tensors).  ``world == 1`` needs no group."""

    def __init__(self, group=None, world: Optional[int] = None, rank: Optional[int] = None,
                 force_collectives: bool = False):
        self.group = group
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world, self.rank = int(world), int(rank)
        # issue the collectives even at world 1 (exercises RCCL + graph capture on one GPU)
        self.force = bool(force_collectives) and dist.is_initialized()

    def exchange(self, send: torch.Tensor) -> torch.Tensor:
        """``out[s]`` = part ``rank`` of rank s's ``send`` (dim 0 split in W equal parts)."""
        if self.world == 1 and not self.force:
            return send
        send = send.contiguous()
        out = torch.empty_like(send)
        dist.all_to_all_single(out, send, group=self.group)
        return out

    def allreduce_sum_(self, flat: torch.Tensor) -> torch.Tensor:
        if self.world > 1 or self.force:
            dist.all_reduce(flat, group=self.group)
        return flat

    def allreduce_mean_(self, flat: torch.Tensor) -> torch.Tensor:
        if self.world > 1 or self.force:
            dist.all_reduce(flat, group=self.group)
            flat.div_(self.world)
        return flat

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src, group=self.group)
        return t


class MrecComm:
    """The ShardComm interface over libmrec's own RCCL communicator (include/mrec.h
    mrec_comm_* / mrec_a2a_* / mrec_allreduce_sum_f32): the exchange a non-torch
    binding would drive, usable from Python for the same sharded step.  The
    128-byte RCCL unique id goes from rank 0 to the others over ``id_channel``
    (a torch.distributed group of any backend, gloo included); world 1 needs none.
    ``close()`` (after every HIP graph that captured its collectives is released)
    destroys the communicator."""

    def __init__(self, world: int = 1, rank: int = 0, id_channel=None):
        lib = _mrec.lib()
        uid = (ctypes.c_char * 128)()
        if rank == 0:
            _mrec.call("mrec_comm_unique_id", ctypes.cast(uid, ctypes.c_void_p))
        if world > 1:
            if not dist.is_initialized():
                raise RuntimeError("MrecComm at world > 1 needs torch.distributed for the id")
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=id_channel)
            ctypes.memmove(uid, box[0], 128)
        h = ctypes.c_void_p()
        _mrec.call("mrec_comm_init", ctypes.cast(uid, ctypes.c_void_p), int(rank), int(world),
                   ctypes.byref(h))
        self._h = h
        self.world, self.rank = int(lib.mrec_comm_world(h)), int(lib.mrec_comm_rank(h))
        self.force = True  # the collectives run even at world 1
        self.group = None

    def exchange(self, send: torch.Tensor) -> torch.Tensor:
        """``out[s]`` = part ``rank`` of rank s's ``send`` (dim 0 in W equal parts)."""
        send = send.contiguous()
        out = torch.empty_like(send)
        per = send.numel() // self.world
        st = _mrec.stream_handle()
        if send.dtype == torch.int32:
            _mrec.call("mrec_a2a_ids", self._h, send.data_ptr(), out.data_ptr(), per, st)
        elif send.dtype == torch.float32:
            _mrec.call("mrec_a2a_rows_bwd", self._h, send.data_ptr(), out.data_ptr(), per, st)
        else:
            _mrec.call("mrec_a2a_rows_fwd", self._h, send.data_ptr(), out.data_ptr(),
                       per * send.element_size(), st)
        return out

    def allreduce_sum_(self, flat: torch.Tensor) -> torch.Tensor:
        if flat.dtype != torch.float32 or not flat.is_contiguous():
            raise ValueError("mrec_allreduce_sum_f32 takes a contiguous fp32 buffer")
        _mrec.call("mrec_allreduce_sum_f32", self._h, flat.data_ptr(), flat.numel(),
                   _mrec.stream_handle())
        return flat

    def allreduce_mean_(self, flat: torch.Tensor) -> torch.Tensor:
        self.allreduce_sum_(flat)
        if self.world > 1:
            flat.div_(self.world)
        return flat

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src)
        return t

    def close(self):
        if self._h:
            _mrec.call("mrec_comm_destroy", self._h)
            self._h = None


def default_cap(batch: int, world: int, rows: Optional[Sequence[int]] = None,
                sigmas: float = 8.0, dedup: bool = False) -> int:
    """Slots per (owner, table), sized for ids spread uniformly over each table: the
    count of a table's ids owned by one rank is Binomial(batch, p) with p the
    largest owner share of the table's rows (ceil(n / W) / n, 1/W for big tables),
    so mean + 8 sd (rounded up to 8) overflows with probability < 1e-14 per (owner,
    table) — at W = 8, B = 4096 that is 688 slots for a mean of 512, where a 2x
    share would move 1.5x the bytes over xGMI in each of the three all-to-alls.
    Skewed ids (Zipf) need a larger ``cap`` (an overflow is raised, never dropped).
    An owner whose exchange view (W * cap entries per table) exceeds one plan
    workgroup's MREC_BWD_MAX_BATCH takes the large-batch path (owner_apply_large)."""
    batch, world = int(batch), int(world)
    if world <= 1:
        return max(1, batch)
    # ``dedup`` (the compact exchange): slots hold DISTINCT ids, so a table's bound is
    # also its owner's expected distinct rows hit (m = ceil(n / W) owned rows, each
    # hit with q = 1 - (1 - 1/n)^B: mean m q + 8 sd) and m itself -- a 1-row table
    # needs one slot, not B
    ns = [int(n) for n in (rows or []) if int(n) > 0]
    if not dedup or not ns:
        shares = [-(-n // world) / n for n in ns]
        p = max(shares + [1.0 / world])
        sd = math.sqrt(batch * p * (1.0 - p))
        cap = int(math.ceil(batch * p + sigmas * sd))
    else:
        cap = 0
        for n in ns:
            m = -(-n // world)
            p = m / n
            look = batch * p + sigmas * math.sqrt(batch * p * (1.0 - p))
            q = -math.expm1(batch * math.log1p(-1.0 / n)) if n > 1 else 1.0
            dist = m * q + sigmas * math.sqrt(m * q * (1.0 - q))
            cap = max(cap, int(math.ceil(min(look, dist, m))))
    cap = (cap + 7) // 8 * 8
    return max(1, min(batch, cap))


def default_cap_rows(batch: int, world: int, rows: Sequence[int], cap: int,
                     sigmas: float = 8.0) -> int:
    """Records per owner part of the compact exchange (all tables together): the
    number of one rank's lookups owned by one rank is a sum over the tables of
    Binomial(batch, p_f), so mean + 8 sd of the SUM (rounded up to 8) -- at W = 8,
    B = 4096, 26 large tables: 14,176 records for a mean of 13,312, where 26
    per-table capacities of 688 would be 17,888 -- bounded by n_tables * cap."""
    batch, world = int(batch), int(world)
    n_tab = max(1, len(rows))
    if world <= 1:
        return max(1, n_tab * min(batch, cap))
    mean = var = 0.0
    for n in rows:
        n = int(n)
        p = (-(-n // world) / n) if n > 0 else 0.0
        mean += batch * p
        var += batch * p * (1.0 - p)
    c = (int(math.ceil(mean + sigmas * math.sqrt(var))) + 7) // 8 * 8
    return max(1, min(c, n_tab * cap))


# ----------------------------------------------------------------------------
# the sharded bank
# ----------------------------------------------------------------------------


class ShardedEmbeddingBank(EmbeddingBank):
    """This rank's shard of F row-sharded tables (same row layout as EmbeddingBank).

    ``category_nums`` are the GLOBAL row counts; local table f holds rows
    ``rank, rank + W, ...`` of global table f.  The update is always the fused
    row-sparse SGD (the table gradient never exists)."""

    def __init__(self, category_nums: Sequence[int], dim: int, comm: ShardComm,
                 with_first_order: bool = False, dtype: torch.dtype = torch.float32,
                 cap: Optional[int] = None, max_batch: int = 4096, device=None):
        W, r = comm.world, comm.rank
        local = [(int(n) - r + W - 1) // W if int(n) > r else 0 for n in category_nums]
        super().__init__([max(n, 0) for n in local], dim, with_first_order, dtype,
                         update="sgd", device=device)
        self.global_rows = [int(n) for n in category_nums]
        self.comm = comm
        self.world, self.rank = W, r
        # the compact exchange's chunks: its per-(owner, wave-group) rank histogram
        # holds (W + 1) * ceil(chunk / 1024) * 16 <= 2048 entries, so large worlds take
        # smaller chunks (W = 16: 7,168 samples; W >= 127 is not supported)
        if W + 1 > 128:
            raise ValueError(f"row sharding supports world sizes up to 127, not {W}")
        cb = int(os.environ.get("MREC_SHARD_CHUNK", type(self).chunk_batch))  # (A/B knob)
        self.chunk_batch = min(cb, 1024 * (128 // (W + 1)))
        # slots per (owner, table[, chunk]): distinct ids of one chunk on the compact
        # exchange, lookups of the whole batch on the slot exchange (which does not
        # chunk); the `compact` setter switches a defaulted cap
        mb = min(int(max_batch), self.chunk_batch)
        self._caps = None if cap is not None else (
            default_cap(mb, W, self.global_rows, dedup=True),
            default_cap(int(max_batch), W, self.global_rows))
        self._max_batch = mb
        self._compact = True
        on = W > 1  # the default exchange: compact at W > 1 (see `compact`)
        self.cap = int(cap) if cap is not None else self._caps[0 if on else 1]
        if self.cap < 1:
            raise ValueError(f"cap = {self.cap} must be >= 1")
        self._flags = None  # device int32 [2] = {overflow, oob}, sticky until checked
        self._global_rows_arr = (ctypes.c_int64 * len(self.global_rows))(*self.global_rows)
        # the compact exchange (one record per distinct id, ABI 19) at world > 1
        # ("always": at world 1 too); False: one slot row per lookup (ABI 14).  At
        # world 1 nothing crosses xGMI and the slot
        # path keeps the step bit-identical to the unsharded bank (the compact path
        # rounds each rank's gradient sum of a bf16 row to bf16 on the wire).
        self._cap_rows = default_cap_rows(mb, W, self.global_rows, self._caps[0]
                                          if self._caps is not None else self.cap)
        self._cap_rows_user = False
        # the dedup bucketize's workgroups per table (mrec_shard_bucketize_dedup_q, ABI
        # 28; a power of two <= 16) and its scratch.  1 by default: 2 or 4 quarters
        # measured no faster at C2's shape (11.9-12.2 us against 11.9 at W = 1; the
        # launch is a chain of id loads, barriers and stores, not of inserts)
        self.dedup_quarters = int(os.environ.get("MREC_DEDUP_QUARTERS", "1"))
        self._dedup_scratch = None

    def dedup_scratch(self, chunks: int) -> torch.Tensor:
        """The quarters' meeting words for ``chunks`` chunks (zeroed once, kept: they
        hold monotonic arrival tickets)."""
        nb = int(_mrec.lib().mrec_shard_dedup_scratch_bytes(self.n_tables, max(1, chunks),
                                                            self.world, self.dedup_quarters))
        if self._dedup_scratch is None or self._dedup_scratch.numel() < nb:
            self._dedup_scratch = torch.zeros(nb, dtype=torch.uint8, device=self.weight.device)
        return self._dedup_scratch

    @property
    def cap_rows(self) -> int:
        """Records per owner part of the compact exchange (default_cap_rows); an
        assigned value is kept when ``compact`` is toggled later."""
        return self._cap_rows

    @cap_rows.setter
    def cap_rows(self, value):
        self._cap_rows = int(value)
        self._cap_rows_user = True

    @property
    def compact(self):
        return self._compact

    @compact.setter
    def compact(self, value):
        """True / "always" / False (see __init__); a defaulted cap follows it (and a
        defaulted cap_rows follows the cap)."""
        self._compact = value
        if self._caps is not None:
            on = value == "always" or (bool(value) and self.world > 1)
            self.cap = self._caps[0] if on else self._caps[1]
            if not self._cap_rows_user:
                self._cap_rows = default_cap_rows(self._max_batch, self.world, self.global_rows,
                                                  self._caps[0])

    @property
    def part(self) -> int:
        """int32 per owner part of the compact ids message: slots, then counts."""
        return self.n_tables * self.cap + self.n_tables

    # a sender's batch past one bucketize workgroup (8192 samples) goes out in
    # chunks, each its own sub-sender: W * chunks parts on the compact exchange
    chunk_batch = 8192

    def chunks(self, batch: int) -> int:
        return max(1, -(-int(batch) // self.chunk_batch))

    def parts(self, batch: int) -> int:
        """Parts of the compact exchange's messages for a batch: world x chunks."""
        return self.world * self.chunks(batch)

    def wire_bytes(self) -> int:
        dt = _mrec.dtype_code(self.weight.dtype)
        return int(_mrec.lib().mrec_shard_wire_bytes(self.dim, int(self.has_w), dt))

    def use_compact(self, batch: int) -> bool:
        """The compact exchange when it is on and mrec_shard_bucketize_dedup_ex takes
        the shape: cap < 65535 (its per-(owner, wave-group) histogram always fits:
        ``chunk_batch`` shrinks with the world size).  Batches past ``chunk_batch``
        go out in chunks.  The slot exchange (compact off) does not chunk: its batch
        must keep (world + 1) * ceil(batch / 1024) * 16 <= 2048 (checked, raised)."""
        on = self.compact == "always" or (bool(self.compact) and self.world > 1)
        return on and self.cap < 65535

    def check_slot_batch(self, batch: int):
        groups = -(-int(batch) // 1024) * 16
        if (self.world + 1) * groups > 2048:
            raise ValueError(
                f"the slot exchange (compact off) takes at most {2048 // 16 // (self.world + 1)}"
                f" x 1024 samples per rank at world {self.world}, not {batch}: use the compact "
                "exchange (ShardedEmbeddingBank.compact = True) or smaller batches")

    @property
    def g_ld(self) -> int:
        return (self.dim + (1 if self.has_w else 0) + 3) // 4 * 4

    def flags(self) -> torch.Tensor:
        if self._flags is None or self._flags.device != self.weight.device:
            self._flags = torch.zeros(2, dtype=torch.int32, device=self.weight.device)
        return self._flags

    def check_flags(self):
        """Raise if any exchange since the last check overflowed its slots or saw an
        out-of-range id (syncs once)."""
        f = self.flags()
        ov, oob = (int(x) for x in f.tolist())
        f.zero_()
        if ov & 1:  # (overflowed lookups also read slot -1, which sets the OOB flag)
            raise RuntimeError(f"row-sharded exchange overflow: more than cap={self.cap} ids of "
                               "one table for one owner in a batch; raise `cap` "
                               "(sharded_tables(cap=...))")
        if ov & 4:
            raise RuntimeError("row-sharded dedup bucketize: a quarter workgroup's wait for "
                               "its siblings timed out (slots of that table are not valid); "
                               "MREC_DEDUP_QUARTERS=1 runs one workgroup per table")
        if ov & 2:
            raise RuntimeError(f"row-sharded compact exchange overflow: more than cap_rows="
                               f"{self.cap_rows} distinct ids for one owner over all tables in a "
                               "batch (their rows were not exchanged and got no update); raise "
                               "`cap_rows` (ShardedEmbeddingBank.cap_rows, default "
                               "default_cap_rows: mean + 8 sd)")
        if oob:
            raise IndexError("index out of range in self")
        super().check_flags()

    # -- global <-> shard ------------------------------------------------------
    @torch.no_grad()
    def load_global_(self, tables: Sequence[torch.Tensor]):
        """Fill the shard from full global tables (each [rows_f, >= dim(+1)])."""
        for f, t in enumerate(tables):
            n = self.category_nums[f]
            if n == 0:
                continue
            src = t[self.rank::self.world]
            o = self.row_offset[f]
            cols = self.dim + (1 if self.has_w else 0)
            self.weight[o:o + n, :cols].copy_(src[:, :cols].to(device=self.weight.device,
                                                                   dtype=self.weight.dtype))
        return self

    @torch.no_grad()
    def gather_global(self, dst: Optional[int] = None,
                      chunk_rows: int = 1 << 22) -> Optional[torch.Tensor]:
        """The full bank in the UNSHARDED layout (``EmbeddingBank(global_rows)``:
        tables concatenated, same row pitch), in HOST memory on rank ``dst`` (every
        rank when None; the others return None).  Per table, chunks of ``chunk_rows``
        global rows: one all_gather of each rank's rows of the chunk, then global row
        i = row i // W of rank i % W -- the GPUs hold one chunk beside their shard,
        never the bank.  Collective: every rank must call it.  (Banks too large for
        one host: IModel.save_weights writes per-rank shard files, checkpoint.py.)"""
        W = self.world
        keep = dst is None or dst == self.rank
        full = (torch.empty(sum(self.global_rows), self.row_stride, dtype=self.weight.dtype)
                if keep else None)
        g_off = 0
        per_chunk = max(1, chunk_rows // W)  # local rows per rank and chunk
        for f, n in enumerate(self.global_rows):
            per = -(-n // W)
            local = self.weight[self.row_offset[f]:self.row_offset[f] + self.category_nums[f]]
            for a in range(0, per, per_chunk):
                b = min(per, a + per_chunk)
                if W == 1:
                    if keep:
                        full[g_off + a:g_off + b] = local[a:b].cpu()
                    continue
                pad = torch.zeros(b - a, self.row_stride, dtype=self.weight.dtype,
                                  device=self.weight.device)
                mine = local[a:min(b, local.shape[0])]
                pad[:mine.shape[0]] = mine
                parts = [torch.empty_like(pad) for _ in range(W)]
                dist.all_gather(parts, pad, group=self.comm.group)
                if keep:
                    # [W, c, stride] -> [c, W, stride]: row j of rank r is global j*W + r
                    inter = torch.stack(parts, 1).reshape((b - a) * W, self.row_stride)
                    lo, hi = a * W, min(n, b * W)
                    full[g_off + lo:g_off + hi] = inter[:hi - lo].cpu()
                del parts, pad
            g_off += n
        return full

    @torch.no_grad()
    def load_global_bank_(self, full: torch.Tensor):
        """Inverse of ``gather_global``: take this rank's rows of a full bank in the
        unsharded layout (e.g. a single-GPU checkpoint's ``embeddings.weight``)."""
        if tuple(full.shape) != (sum(self.global_rows), self.row_stride):
            raise ValueError(f"full bank shape {tuple(full.shape)} != "
                             f"({sum(self.global_rows)}, {self.row_stride})")
        offs = [0]
        for n in self.global_rows:
            offs.append(offs[-1] + n)
        return self.load_global_([full[offs[f]:offs[f + 1]] for f in range(len(self.global_rows))])

    def local_rows_of(self, f: int) -> torch.Tensor:
        """Global ids of this shard's rows of table f."""
        return torch.arange(self.rank, self.global_rows[f], self.world)

    def extra_repr(self) -> str:
        return (super().extra_repr() + f", world={self.world}, rank={self.rank}, cap={self.cap}, "
                f"cap_rows={self.cap_rows}, compact={self.compact}")


_ACTIVE: List[tuple] = []


@contextlib.contextmanager
def sharded_tables(comm: ShardComm, cap: Optional[int] = None, max_batch: int = 4096):
    """Models built inside this context get ``ShardedEmbeddingBank`` tables
    (no rank ever materialises a full table)."""
    _ACTIVE.append((comm, cap, max_batch))
    try:
        yield
    finally:
        _ACTIVE.pop()


def make_bank(category_nums, dim, with_first_order=False, dtype=torch.float32, device=None):
    """EmbeddingBank factory used by the models' ``_init_weights``."""
    if _ACTIVE:
        comm, cap, max_batch = _ACTIVE[-1]
        return ShardedEmbeddingBank(category_nums, dim, comm, with_first_order, dtype, cap,
                                    max_batch, device)
    return EmbeddingBank(category_nums, dim, with_first_order=with_first_order, dtype=dtype,
                         device=device)


# ----------------------------------------------------------------------------
# GPU phases (each one libmrec call; usable on their own, e.g. to drive several
# simulated ranks in one process)
# ----------------------------------------------------------------------------


def shard_bucketize(bank: ShardedEmbeddingBank, ids: Sequence[torch.Tensor]):
    """-> (send_ids [W, F, cap] int32, pos [F, B] int32)."""
    F, W, cap = bank.n_tables, bank.world, bank.cap
    B = ids[0].shape[0]
    dev = bank.weight.device
    send = torch.empty(W, F, cap, dtype=torch.int32, device=dev)
    pos = torch.empty(F, B, dtype=torch.int32, device=dev)
    fl = bank.flags()
    _mrec.call("mrec_shard_bucketize", _mrec.IdsDesc(ids).ref(), F, bank._global_rows_arr, B, W,
               cap, send.data_ptr(), pos.data_ptr(), fl.data_ptr(), fl.data_ptr() + 4,
               _mrec.stream_handle())
    return send, pos


def shard_gather(bank: ShardedEmbeddingBank, recv_ids: torch.Tensor) -> torch.Tensor:
    """Owner: rows of the received ids -> [W*F*cap, row_stride] (bank dtype)."""
    n = recv_ids.numel()
    out = torch.empty(n, bank.row_stride, dtype=bank.weight.dtype, device=bank.weight.device)
    _mrec.call("mrec_shard_gather", bank.desc().ref(), recv_ids.data_ptr(), bank.world, bank.cap,
               out.data_ptr(), _mrec.stream_handle())
    return out


def shard_bucketize_dedup(bank: ShardedEmbeddingBank, ids: Sequence[torch.Tensor]):
    """-> (send_ids [W, C * (F*cap + F)] int32: distinct ids per (owner, table) +
    counts for each of the C chunks of the batch (bank.chunks), pos [F, B] int32:
    the slot of every lookup in the W * C parts' slot rows)."""
    F, W, cap = bank.n_tables, bank.world, bank.cap
    B = ids[0].shape[0]
    C = bank.chunks(B)
    dev = bank.weight.device
    send = torch.empty(W, C * bank.part, dtype=torch.int32, device=dev)
    pos = torch.empty(F, B, dtype=torch.int32, device=dev)
    fl = bank.flags()
    H = bank.dedup_quarters
    scratch = bank.dedup_scratch(C) if H > 1 else None
    _mrec.call("mrec_shard_bucketize_dedup_q", _mrec.IdsDesc(ids).ref(), F,
               bank._global_rows_arr, B, W, cap, bank.chunk_batch, H, _mrec.ptr(scratch),
               scratch.numel() if scratch is not None else 0, send.data_ptr(), pos.data_ptr(),
               fl.data_ptr(), fl.data_ptr() + 4, _mrec.stream_handle())
    return send, pos


def shard_gather_wire(bank: ShardedEmbeddingBank, recv_ids: torch.Tensor,
                      plan_job=None, pref: Optional[torch.Tensor] = None,
                      parts: Optional[int] = None) -> torch.Tensor:
    """Owner: one record per received distinct id -> [W, cap_rows * record] bytes.
    ``plan_job`` (owner_plan_job) runs the owner's backward plan over the same ids in
    leading workgroups of the launch; ``pref`` (int32 [W, n_tables]) receives each
    part's table prefixes (mrec_shard_gather_wire_ex), which address the gradient
    records the senders return (owner_apply_wire).  ``parts``: W * chunks."""
    P, rb = parts or bank.world, bank.wire_bytes()
    wire = torch.empty(P, bank.cap_rows * rb, dtype=torch.uint8, device=bank.weight.device)
    fl = bank.flags()
    _mrec.call("mrec_shard_gather_wire_ex", bank.desc().ref(), recv_ids.data_ptr(), P, bank.cap,
               bank.cap_rows, wire.data_ptr(), _mrec.ptr(pref), fl.data_ptr(),
               ctypes.byref(plan_job) if plan_job is not None else None, _mrec.stream_handle())
    return wire


def shard_wire_unpack(bank: ShardedEmbeddingBank, wire: torch.Tensor, hdr: torch.Tensor,
                      slots: torch.Tensor, to_f32: bool = False,
                      zero: Optional[torch.Tensor] = None, parts: Optional[int] = None,
                      pref: Optional[torch.Tensor] = None):
    """Records -> slot rows [W*F*cap, ...] (``hdr``: the ids message whose counts
    describe ``wire``); ``zero``: the same rows of a second buffer are cleared;
    ``pref`` (int32 [parts, n_tables]) receives each part's table prefixes -- the
    record layout sender_grad_records writes the gradients in."""
    fl = bank.flags()
    _mrec.call("mrec_shard_wire_unpack_ex", wire.data_ptr(), bank.wire_bytes(), hdr.data_ptr(),
               parts or bank.world, bank.n_tables, bank.cap, bank.cap_rows, slots.data_ptr(),
               slots.stride(0) * slots.element_size(), int(to_f32), _mrec.ptr(zero),
               zero.stride(0) * zero.element_size() if zero is not None else 0, _mrec.ptr(pref),
               fl.data_ptr(), _mrec.stream_handle())
    return slots


def shard_wire_pack(bank: ShardedEmbeddingBank, slots: torch.Tensor, hdr: torch.Tensor,
                    parts: Optional[int] = None):
    """Slot rows (the table dtype) -> records [W * chunks, cap_rows * record] bytes."""
    P, rb = parts or bank.world, bank.wire_bytes()
    wire = torch.empty(P, bank.cap_rows * rb, dtype=torch.uint8, device=bank.weight.device)
    fl = bank.flags()
    _mrec.call("mrec_shard_wire_pack", slots.data_ptr(), slots.stride(0) * slots.element_size(),
               rb, hdr.data_ptr(), P, bank.n_tables, bank.cap, bank.cap_rows, wire.data_ptr(),
               fl.data_ptr(), _mrec.stream_handle())
    return wire


def sender_plan_job(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor):
    """The sender's backward plan over its lookups' slots (the slot rows seen as a
    bank, ids = pos) as a job for the interaction launch -> (job, (ws, bytes), keep)."""
    F = bank.n_tables
    B = pos.shape[1]
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, B)
    ws = torch.empty(wsb, dtype=torch.uint8, device=bank.weight.device)
    rdesc = remote_desc(bank, rows_recv)
    rdesc.ref()
    idd = _mrec.IdsDesc([pos[f] for f in range(F)])
    fl = bank.flags()
    job = _mrec.PlanJob(ctypes.pointer(rdesc.struct), ctypes.pointer(idd.struct), B, ws.data_ptr(),
                        wsb, fl.data_ptr() + 4, None)
    return job, (ws, wsb), (rdesc, idd, pos, rows_recv)


def sender_plan(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor):
    """sender_plan_job as its own launch (batches above MREC_BWD_HASH_MAX_BATCH)."""
    F = bank.n_tables
    B = pos.shape[1]
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, B)
    ws = torch.empty(wsb, dtype=torch.uint8, device=bank.weight.device)
    fl = bank.flags()
    _mrec.call("mrec_emb_bwd_plan", remote_desc(bank, rows_recv).ref(),
               _mrec.IdsDesc([pos[f] for f in range(F)]).ref(), B, ws.data_ptr(), wsb,
               fl.data_ptr() + 4, None, _mrec.stream_handle())
    return ws, wsb


def sender_plans(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor):
    """sender_plan per chunk of bank.chunk_batch samples (a chunk's lookups address
    only its own parts' slots, so each is summed on its own) -> [(s0, n, plan)]."""
    B = pos.shape[1]
    cb = bank.chunk_batch
    out = []
    for s0 in range(0, B, cb):
        n = min(cb, B - s0)
        out.append((s0, n, sender_plan(bank, rows_recv, pos[:, s0:s0 + n])))
    return out or [(0, 0, sender_plan(bank, rows_recv, pos))]


def sender_grad_sums(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor,
                     plan, gsum: torch.Tensor, dx=None, dfm=None, fm_sum=None, x0=None, dw=None):
    """Sender: per slot, the sum of its lookups' gradient rows (fp32, ascending
    sample order; stored in the table dtype = the wire format) into ``gsum``
    (slot rows, zeroed by the unpack).  The deferred MLP weight-gradient
    reductions ride along this launch."""
    ws, wsb = plan
    B = pos.shape[1]
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    rdesc = remote_desc(bank, rows_recv)
    _mrec.call("mrec_emb_bwd_apply_ex", rdesc.ref(), B, ws.data_ptr(), wsb,
               _mrec.ptr(dx), _mrec.dtype_code(dx.dtype) if dx is not None else _mrec.F32,
               dx.stride(0) if dx is not None else 0, _mrec.ptr(dfm), _mrec.ptr(fm_sum),
               _mrec.ptr(x0), _mrec.dtype_code(x0.dtype) if x0 is not None else _mrec.F32,
               x0.stride(0) if x0 is not None else 0, _mrec.ptr(dw), _mrec.BWD_DENSE_GRAD, 0.0,
               0, None, gsum.data_ptr(), len(jobs), arr, _mrec.stream_handle())
    del jobs
    return gsum


def sender_grad_records(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor,
                        plan, spref: torch.Tensor, parts: Optional[int] = None, dx=None, dfm=None,
                        fm_sum=None, x0=None, dw=None) -> torch.Tensor:
    """sender_grad_sums + shard_wire_pack in ONE launch (mrec_emb_bwd_apply_rec, ABI
    26): each slot's sum goes straight into its wire record (``spref``: the part
    prefixes shard_wire_unpack wrote) -> [parts, cap_rows * record] bytes, the same
    bytes the pack of a zeroed sum buffer gives.  Hash-layout plans only (B <=
    MREC_BWD_HASH_MAX_BATCH); the deferred MLP reductions ride along."""
    ws, wsb = plan
    B = pos.shape[1]
    P, rb = parts or bank.world, bank.wire_bytes()
    wire = torch.empty(P, bank.cap_rows * rb, dtype=torch.uint8, device=bank.weight.device)
    out = _mrec.GradRecords(wire.data_ptr(), rb, spref.data_ptr(), bank.cap, bank.cap_rows)
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    rdesc = remote_desc(bank, rows_recv)
    _mrec.call("mrec_emb_bwd_apply_rec", rdesc.ref(), B, ws.data_ptr(), wsb,
               _mrec.ptr(dx), _mrec.dtype_code(dx.dtype) if dx is not None else _mrec.F32,
               dx.stride(0) if dx is not None else 0, _mrec.ptr(dfm), _mrec.ptr(fm_sum),
               _mrec.ptr(x0), _mrec.dtype_code(x0.dtype) if x0 is not None else _mrec.F32,
               x0.stride(0) if x0 is not None else 0, _mrec.ptr(dw), ctypes.byref(out),
               len(jobs), arr, _mrec.stream_handle())
    del jobs
    return wire


def remote_desc(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor) -> _mrec.BankDesc:
    """The received rows seen as a bank: F tables over the same buffer, each table's
    'id' being the slot index (pos)."""
    F = bank.n_tables
    n = rows_recv.shape[0]
    return _mrec.BankDesc(rows_recv, [0] * F, [n] * F, bank.dim, bank.has_w)


def owner_plan_job(bank: ShardedEmbeddingBank, recv_ids: torch.Tensor, part: int = 0,
                   parts: Optional[int] = None):
    """The owner's backward plan as a job for the interaction launch (hash layout
    over the padded exchange view, <= MREC_BWD_MAX_BATCH entries; ``part``: int32
    per owner part of the ids message, 0 = n_tables * cap) ->
    (job, (ws, ws_bytes), keep-alive)."""
    F, W, cap = bank.n_tables, parts or bank.world, bank.cap
    n = W * cap
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=bank.weight.device)
    desc = bank.desc()
    desc.ref()
    idd = _mrec.IdsDesc.exchange_view(recv_ids, F, cap, part)
    fl = bank.flags()
    job = _mrec.PlanJob(ctypes.pointer(desc.struct), ctypes.pointer(idd.struct), n, ws.data_ptr(),
                        wsb, fl.data_ptr() + 4, bank.step_counter().data_ptr())
    return job, (ws, wsb), (desc, idd, recv_ids)


def records_direct(bank: ShardedEmbeddingBank) -> bool:
    """Whether the interaction reads the received records itself
    (mrec_interact_fwd_rec: bf16 64-B slot rows; a lazy-Adam bank's rows were caught
    up by the owner's gather) instead of after an unpack launch; MREC_SHARD_UNPACK=1
    forces the unpack (A/B)."""
    return (bank.weight.dtype == torch.bfloat16 and bank.row_stride * 2 == 64
            and os.environ.get("MREC_SHARD_UNPACK") != "1")


def shard_interact(bank: ShardedEmbeddingBank, rows_recv: torch.Tensor, pos: torch.Tensor,
                   dense, dense_w, bias, fm2: bool, first_order: bool, x0_cols: int, x0_dtype,
                   plan_job=None, rec=None):
    """Sender: mrec_interact_fwd over the received rows (ids = slots) ->
    (x0 or None, logit, fm_sum or None).  ``plan_job`` (owner_plan_job) runs the
    owner's backward plan in leading workgroups of the same launch.  ``rec``: a
    WireRows -- the rows come from the received records (mrec_interact_fwd_rec),
    which the same launch also writes into ``rows_recv`` (the unpack's bytes)."""
    B = pos.shape[1]
    dev = bank.weight.device
    rdesc = remote_desc(bank, rows_recv)
    n_dense = 0 if dense is None else dense.shape[1]
    flags = (_mrec.INTERACT_FM2 if fm2 else 0) | (_mrec.INTERACT_FIRST_ORDER if first_order else 0)
    x0 = torch.empty(B, x0_cols, dtype=x0_dtype, device=dev) if x0_cols else None
    logit = torch.empty(B, dtype=torch.float32, device=dev)
    fm_sum = torch.empty(B, bank.dim, dtype=torch.float32, device=dev) if fm2 else None
    fl = bank.flags()
    if B:
        args = (rdesc.ref(), _mrec.IdsDesc([pos[f] for f in range(bank.n_tables)]).ref(), B,
                _mrec.ptr(dense), n_dense, dense.stride(0) if dense is not None else 0,
                _mrec.ptr(dense_w), _mrec.ptr(bias), flags, _mrec.ptr(x0),
                _mrec.dtype_code(x0_dtype), x0.stride(0) if x0 is not None else 0,
                int(x0_cols), logit.data_ptr(), _mrec.ptr(fm_sum), fl.data_ptr() + 4,
                ctypes.byref(plan_job) if plan_job is not None else None)
        if rec is not None:
            _mrec.call("mrec_interact_fwd_rec", *args, ctypes.byref(rec), _mrec.stream_handle())
        else:
            _mrec.call("mrec_interact_fwd_ex", *args, _mrec.stream_handle())
    return x0, logit, fm_sum


def owner_plan(bank: ShardedEmbeddingBank, recv_ids: torch.Tensor, part: int = 0,
               parts: Optional[int] = None):
    """Sorted-segment plan of the owner's received ids (padding skipped; ``part``
    as in owner_plan_job)."""
    F, W, cap = bank.n_tables, parts or bank.world, bank.cap
    n = W * cap
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=bank.weight.device)
    desc = _mrec.IdsDesc.exchange_view(recv_ids, F, cap, part)
    fl = bank.flags()
    _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), desc.ref(), n, ws.data_ptr(), wsb,
               fl.data_ptr() + 4, bank.step_counter().data_ptr(), _mrec.stream_handle())
    return ws, wsb


def shard_lookup_grad(bank: ShardedEmbeddingBank, pos: torch.Tensor, batch: int, dx=None,
                      dfm=None, fm_sum=None, x0=None, dw=None) -> torch.Tensor:
    """Sender: per-lookup gradient rows at their slots -> [W*F*cap, g_ld] fp32."""
    F, W, cap = bank.n_tables, bank.world, bank.cap
    g = torch.empty(W * F * cap, bank.g_ld, dtype=torch.float32, device=bank.weight.device)
    _mrec.call("mrec_shard_lookup_grad", batch, F, bank.dim, int(bank.has_w), pos.data_ptr(),
               _mrec.ptr(dx), _mrec.dtype_code(dx.dtype) if dx is not None else _mrec.F32,
               dx.stride(0) if dx is not None else 0, _mrec.ptr(dfm), _mrec.ptr(fm_sum),
               _mrec.ptr(x0), _mrec.dtype_code(x0.dtype) if x0 is not None else _mrec.F32,
               x0.stride(0) if x0 is not None else 0, _mrec.ptr(dw), g.data_ptr(), g.shape[1],
               _mrec.stream_handle())
    return g


def owner_apply(bank: ShardedEmbeddingBank, plan, g_recv: torch.Tensor,
                lr: Optional[float] = None, grad: Optional[torch.Tensor] = None):
    """Owner: fixed-order segment sums of the received gradient rows + the fused
    update.  The rows arrive summed over the W ranks' batches; each rank's loss is
    its own batch mean, so SGD steps with lr / W and a fused optimizer sees the
    sum scaled by 1 / W (its grad_scale): the data-parallel mean gradient.  An
    explicit ``lr`` runs plain SGD with exactly that step (kernel tests)."""
    ws, wsb = plan
    F, W, cap = bank.n_tables, bank.world, bank.cap
    if grad is not None:  # the summed gradient into a dense buffer (kernel tests)
        mode, lr = _mrec.BWD_DENSE_GRAD, 0.0
    elif lr is not None:
        mode = (_mrec.BWD_SGD_SR if (bank.stochastic_rounding and
                                     bank.weight.dtype == torch.bfloat16) else _mrec.BWD_SGD)
    else:
        mode, lr = bank.apply_mode()
        if mode in (_mrec.BWD_SGD, _mrec.BWD_SGD_SR):
            lr = lr / W
    # deferred MLP weight-gradient reductions ride along this launch
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    _mrec.call("mrec_emb_bwd_apply_given", bank.desc().ref(), W * cap, ws.data_ptr(), wsb,
               None, _mrec.F32, 0, None, None, None, _mrec.F32, 0, None, g_recv.data_ptr(),
               g_recv.shape[1], cap, F * cap, mode, float(lr), bank.next_seed(),
               bank.step_counter().data_ptr(), _mrec.ptr(grad), len(jobs), arr,
               _mrec.stream_handle())
    del jobs


def owner_apply_wire(bank: ShardedEmbeddingBank, plan, wire_g: torch.Tensor, pref: torch.Tensor,
                     lr: Optional[float] = None, grad: Optional[torch.Tensor] = None,
                     parts: Optional[int] = None, sgd=None):
    """owner_apply reading the received gradient records in place
    (mrec_emb_bwd_apply_wire: no unpack to fp32 slots; same sums and update).
    ``sgd``: (device table, workgroups) of mrec_sgd_table_build -- the data-parallel
    dense SGD rides in the same launch (mrec_emb_bwd_apply_wire_sgd, ABI 28)."""
    ws, wsb = plan
    F, W, cap = bank.n_tables, parts or bank.world, bank.cap
    mode, lr = _owner_mode(bank, lr, grad)
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    args = (bank.desc().ref(), W * cap, ws.data_ptr(), wsb, wire_g.data_ptr(), bank.wire_bytes(),
            _mrec.dtype_code(bank.weight.dtype), pref.data_ptr(), bank.cap_rows, cap, F * cap, mode,
            float(lr), bank.next_seed(), bank.step_counter().data_ptr(), _mrec.ptr(grad),
            len(jobs), arr)
    if sgd is not None:
        _mrec.call("mrec_emb_bwd_apply_wire_sgd", *args, sgd[0].data_ptr(), int(sgd[1]),
                   _mrec.stream_handle())
    else:
        _mrec.call("mrec_emb_bwd_apply_wire", *args, _mrec.stream_handle())
    del jobs


def _owner_mode(bank: ShardedEmbeddingBank, lr, grad):
    if grad is not None:
        return _mrec.BWD_DENSE_GRAD, 0.0
    if lr is not None:
        return (_mrec.BWD_SGD_SR if (bank.stochastic_rounding and
                                     bank.weight.dtype == torch.bfloat16) else _mrec.BWD_SGD), lr
    mode, lr = bank.apply_mode()
    if mode in (_mrec.BWD_SGD, _mrec.BWD_SGD_SR):
        lr = lr / bank.world
    return mode, lr


def owner_view_fits_hash(bank: ShardedEmbeddingBank, parts: Optional[int] = None) -> bool:
    """The owner's exchange view (parts x cap entries per table, parts = W x chunks)
    fits the hash / sorted plan of one workgroup per table; larger views (big W *
    cap: Zipf ids, large batches) take the large-batch path with given gradients
    (owner_apply_large)."""
    return (parts or bank.world) * bank.cap <= _mrec.BWD_MAX_BATCH


def owner_apply_large(bank: ShardedEmbeddingBank, recv_ids: torch.Tensor, part: int,
                      g_occ: Optional[torch.Tensor] = None, wire_g: Optional[torch.Tensor] = None,
                      pref: Optional[torch.Tensor] = None, lr: Optional[float] = None,
                      grad: Optional[torch.Tensor] = None, parts: Optional[int] = None):
    """Owner: the large-batch bucketed plan over the received ids' exchange view
    (W * cap entries per table, padding skipped) and one update per row from the
    GIVEN gradients -- the slot exchange's fp32 slots (``g_occ``) or the compact
    exchange's records (``wire_g`` + ``pref``) -- in ONE call
    (mrec_emb_bwd_large_fused_given, ABI 25).  Rows hit <= 16 times are summed in
    entry order (= sender rank order, as the hash path), hotter rows in the
    order-free 64-bit fixed point."""
    F, W, cap = bank.n_tables, parts or bank.world, bank.cap
    n = W * cap
    mode, lr = _owner_mode(bank, lr, grad)
    ws = _large_ws_for(bank, n)
    idd = _mrec.IdsDesc.exchange_view(recv_ids, F, cap, part)
    g = _mrec.GivenGrads()
    g.chunk = cap
    if g_occ is not None:
        g.g_occ, g.g_ld, g.chunk_stride = g_occ.data_ptr(), g_occ.shape[1], F * cap
    else:
        g.wire, g.rec_bytes = wire_g.data_ptr(), bank.wire_bytes()
        g.wire_dtype, g.pref, g.cap_rows = (_mrec.dtype_code(bank.weight.dtype), pref.data_ptr(),
                                            bank.cap_rows)
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    fl = bank.flags()
    _mrec.call("mrec_emb_bwd_large_fused_given", bank.desc().ref(), idd.ref(), n, ws.data_ptr(),
               ws.numel(), fl.data_ptr() + 4, ctypes.byref(g), mode, float(lr), bank.next_seed(),
               bank.step_counter().data_ptr(), _mrec.ptr(grad), len(jobs), arr,
               _mrec.stream_handle())
    del jobs


def _large_ws_for(bank: ShardedEmbeddingBank, n: int) -> torch.Tensor:
    """The bank's large-batch workspace for exchange views of n entries per table
    (zeroed once; every call leaves its zero region zero)."""
    from pytorchrec_amd.embedding import _large_ws
    return _large_ws(bank, n)


# ----------------------------------------------------------------------------
# autograd (GPU)
# ----------------------------------------------------------------------------


class _CompactInteractFn(torch.autograd.Function):
    """The compact exchange (module docstring): distinct ids out, one record per
    distinct row back, one summed gradient per distinct row to the owners.  A batch
    past 8192 samples goes out as C chunks (sub-senders): every message has W * C
    parts, the sender plans and sums each chunk's lookups on their own."""

    @staticmethod
    def forward(ctx, dense_w, bias, trigger, bank: ShardedEmbeddingBank, ids, dense, fm2: bool,
                first_order: bool, x0_cols: int, x0_dtype):
        B = ids[0].shape[0]
        dev = bank.weight.device
        comm = bank.comm
        P = bank.parts(B)
        send, pos = shard_bucketize_dedup(bank, ids)
        recv = comm.exchange(send)
        train = trigger is not None
        # the owner's backward plan rides in the gather launch (same received ids);
        # a view past one plan workgroup takes the large path in the backward
        ojob_ok = train and owner_view_fits_hash(bank, P)
        ojob, oplan, okeep = (owner_plan_job(bank, recv, bank.part, P) if ojob_ok
                              else (None, None, None))
        pref = (torch.empty(P, bank.n_tables, dtype=torch.int32, device=dev)
                if train else None)
        wire = comm.exchange(shard_gather_wire(bank, recv, plan_job=ojob, pref=pref, parts=P))
        del okeep
        n = P * bank.n_tables * bank.cap
        rows_recv = torch.empty(n, bank.row_stride, dtype=bank.weight.dtype, device=dev)
        fuse = train and B <= _mrec.BWD_HASH_MAX_BATCH
        # one chunk in the hash layout: the backward writes the gradient records
        # directly (sender_grad_records); else sums into zeroed slot rows + a pack
        spref = torch.empty(P, bank.n_tables, dtype=torch.int32, device=dev) if fuse else None
        gsum = torch.empty_like(rows_recv) if train and not fuse else None
        # the interaction reads the records itself (and leaves the unpack's slot rows
        # behind for the backward) unless a zeroed sum buffer is needed too
        direct = gsum is None and records_direct(bank) and P * bank.n_tables <= 8192
        rec = None
        if direct:
            rec = _mrec.WireRows(wire.data_ptr(), bank.wire_bytes(), send.data_ptr(), P, bank.cap,
                                 bank.cap_rows, _mrec.ptr(spref), bank.flags().data_ptr())
        else:
            shard_wire_unpack(bank, wire, send, rows_recv, zero=gsum, parts=P, pref=spref)
        job, splan, keep = (sender_plan_job(bank, rows_recv, pos) if fuse
                            else (None, None, None))
        x0, logit, fm_sum = shard_interact(bank, rows_recv, pos, dense, dense_w, bias, fm2,
                                           first_order, x0_cols, x0_dtype, plan_job=job, rec=rec)
        del keep
        splans = [(0, B, splan)] if fuse else None
        if train and not fuse:
            splans = sender_plans(bank, rows_recv, pos)
        if train and oplan is None and owner_view_fits_hash(bank, P):
            oplan = owner_plan(bank, recv, bank.part, P)
        if bank.check_ids:
            bank.check_flags()
        ctx.bank, ctx.B, ctx.P = bank, B, P
        ctx.splans, ctx.oplan = splans, oplan
        ctx.fm2, ctx.first_order = fm2, first_order
        ctx.has_dense_w, ctx.has_bias = dense_w is not None, bias is not None
        ctx.dense_w, ctx.bias = dense_w, bias
        ctx.pref, ctx.spref = pref, spref
        ctx.save_for_backward(x0, fm_sum, dense, pos, send, recv, rows_recv, gsum)
        if x0 is None:
            return logit
        return x0, logit

    @staticmethod
    def backward(ctx, *grads):
        if len(grads) == 2:
            dx0, dlogit = grads
        else:
            dx0, dlogit = None, grads[0]
        x0, fm_sum, dense, pos, send, recv, rows_recv, gsum = ctx.saved_tensors
        bank = ctx.bank
        if dlogit is not None:
            dlogit = dlogit.contiguous().float()
        dfm = dlogit if (ctx.fm2 and dlogit is not None) else None
        dw = dlogit if (ctx.first_order and dlogit is not None) else None
        if dx0 is not None:
            dx0 = dx0.contiguous()
        if ctx.splans is not None:
            if ctx.spref is not None:  # one hash-layout chunk: records written directly
                (_, _, splan), = ctx.splans
                wire_g = sender_grad_records(bank, rows_recv, pos, splan, ctx.spref, parts=ctx.P,
                                             dx=dx0, dfm=dfm, fm_sum=fm_sum,
                                             x0=x0 if dfm is not None else None, dw=dw)
            else:
                for s0, n_c, splan in ctx.splans:  # each chunk's lookups (disjoint slots)
                    sl = (lambda t: None if t is None else t[s0:s0 + n_c])  # noqa: E731
                    sender_grad_sums(bank, rows_recv, pos[:, s0:s0 + n_c], splan, gsum,
                                     dx=sl(dx0), dfm=sl(dfm), fm_sum=sl(fm_sum),
                                     x0=sl(x0) if dfm is not None else None, dw=sl(dw))
                wire_g = shard_wire_pack(bank, gsum, send, parts=ctx.P)
            wire_g = bank.comm.exchange(wire_g)
            # the owner reads the gradient records in place (no unpack launch); a
            # data-parallel model's dense SGD rides in the same launch when the flat
            # gradient is complete here (IModel._dp_inline_sgd: its all-reduce first)
            if ctx.oplan is not None:
                hook = getattr(bank, "dp_inline_sgd", None)
                sgd = hook() if hook is not None else None
                owner_apply_wire(bank, ctx.oplan, wire_g, ctx.pref, parts=ctx.P, sgd=sgd)
            else:
                owner_apply_large(bank, recv, bank.part, wire_g=wire_g, pref=ctx.pref,
                                  parts=ctx.P)
        g_dense_w, g_bias = _dense_first_order_grads(ctx, dlogit, dense)
        return g_dense_w, g_bias, None, None, None, None, None, None, None, None


class _ShardedInteractFn(torch.autograd.Function):
    """The slot exchange of ABI 14 (one row / fp32 gradient per lookup):
    ``ShardedEmbeddingBank.compact = False`` (and shapes the compact bucketize
    does not take, ShardedEmbeddingBank.use_compact)."""

    @staticmethod
    def forward(ctx, dense_w, bias, trigger, bank: ShardedEmbeddingBank, ids, dense, fm2: bool,
                first_order: bool, x0_cols: int, x0_dtype):
        B = ids[0].shape[0]
        dev = bank.weight.device
        comm = bank.comm
        send_ids, pos = shard_bucketize(bank, ids)
        recv_ids = comm.exchange(send_ids)
        rows_recv = comm.exchange(shard_gather(bank, recv_ids))
        train = trigger is not None
        # the owner's plan rides in the interaction launch when its exchange view fits
        # one plan workgroup per table; else the large path in the backward
        job, plan, keep = (owner_plan_job(bank, recv_ids) if train and owner_view_fits_hash(bank)
                           else (None, None, None))
        x0, logit, fm_sum = shard_interact(bank, rows_recv, pos, dense, dense_w, bias, fm2,
                                           first_order, x0_cols, x0_dtype, plan_job=job)
        del keep
        if bank.check_ids:
            bank.check_flags()
        ctx.bank, ctx.B, ctx.plan, ctx.train = bank, B, plan, train
        ctx.recv_ids = recv_ids if train and plan is None else None
        ctx.fm2, ctx.first_order = fm2, first_order
        ctx.has_dense_w, ctx.has_bias = dense_w is not None, bias is not None
        ctx.dense_w, ctx.bias = dense_w, bias
        ctx.save_for_backward(x0, fm_sum, dense, pos)
        if x0 is None:
            return logit
        return x0, logit

    @staticmethod
    def backward(ctx, *grads):
        if len(grads) == 2:
            dx0, dlogit = grads
        else:
            dx0, dlogit = None, grads[0]
        x0, fm_sum, dense, pos = ctx.saved_tensors
        bank = ctx.bank
        if dlogit is not None:
            dlogit = dlogit.contiguous().float()
        dfm = dlogit if (ctx.fm2 and dlogit is not None) else None
        dw = dlogit if (ctx.first_order and dlogit is not None) else None
        if dx0 is not None:
            dx0 = dx0.contiguous()
        if ctx.train:
            g_send = shard_lookup_grad(bank, pos, ctx.B, dx=dx0, dfm=dfm, fm_sum=fm_sum,
                                       x0=x0 if dfm is not None else None, dw=dw)
            g_recv = bank.comm.exchange(g_send)
            if ctx.plan is not None:
                owner_apply(bank, ctx.plan, g_recv)
            else:
                owner_apply_large(bank, ctx.recv_ids, 0, g_occ=g_recv)
        g_dense_w, g_bias = _dense_first_order_grads(ctx, dlogit, dense)
        return g_dense_w, g_bias, None, None, None, None, None, None, None, None


# ----------------------------------------------------------------------------
# CPU restatement of the same protocol (gloo; the multi-process tests)
# ----------------------------------------------------------------------------


def cpu_bucketize(bank: ShardedEmbeddingBank, ids: Sequence[torch.Tensor]):
    F, W, cap = bank.n_tables, bank.world, bank.cap
    B = ids[0].shape[0]
    send = torch.full((W, F, cap), -1, dtype=torch.int32)
    pos = torch.empty(F, B, dtype=torch.int32)
    for f, t in enumerate(ids):
        t = t.long()
        if t.numel() and (int(t.min()) < 0 or int(t.max()) >= bank.global_rows[f]):
            raise IndexError("index out of range in self")
        owner = t % W
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=W)
        starts = torch.cumsum(counts, 0) - counts
        slot = torch.empty(B, dtype=torch.long)
        slot[order] = torch.arange(B) - starts[owner[order]]
        if B and int(slot.max()) >= cap:
            raise RuntimeError(f"row-sharded exchange overflow: more than cap={cap} ids of one "
                               "table for one owner in a batch; raise cap")
        send[owner, f, slot] = (t // W).to(torch.int32)
        pos[f] = ((owner * F + f) * cap + slot).to(torch.int32)
    return send, pos


def dedup_quarter(ids: torch.Tensor, quarters: int) -> torch.Tensor:
    """The dedup bucketize's quarter of each id (shard.hip dedup_quarter):
    ((id * 0x9e3779b1) mod 2^32) >> (32 - log2 quarters)."""
    lg = max(0, int(quarters).bit_length() - 1)
    if lg == 0:
        return torch.zeros_like(ids, dtype=torch.long)
    return ((ids.long() * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - lg)


def cpu_bucketize_dedup(bank: ShardedEmbeddingBank, ids: Sequence[torch.Tensor]):
    """CPU restatement of mrec_shard_bucketize_dedup(_ex): per (owner, table) the
    distinct ids in the order of their first lookup, every lookup's slot, the
    counts header, for each chunk of bank.chunk_batch samples (sub-sender c of owner
    o's part o * C + c) -> (send [W, C * (F*cap + F)] int32, pos [F, B] int32)."""
    F, W, cap = bank.n_tables, bank.world, bank.cap
    B = ids[0].shape[0]
    C = bank.chunks(B)
    send = torch.full((W, C, bank.part), -1, dtype=torch.int32)
    pos = torch.empty(F, B, dtype=torch.int32)
    for c in range(C):
        s0 = c * bank.chunk_batch
        n = min(bank.chunk_batch, B - s0)
        ar = torch.arange(n)
        for f, t in enumerate(ids):
            t = t[s0:s0 + n].long()
            if t.numel() and (int(t.min()) < 0 or int(t.max()) >= bank.global_rows[f]):
                raise IndexError("index out of range in self")
            owner = t % W
            uniq, inv = torch.unique(t, return_inverse=True)
            first = torch.full((uniq.numel(),), n, dtype=torch.long)
            first.scatter_reduce_(0, inv, ar, reduce="amin")
            rep = first[inv] == ar
            slot_u = torch.empty(uniq.numel(), dtype=torch.long)
            quarter = dedup_quarter(t, getattr(bank, "dedup_quarters", 1))
            for o in range(W):
                r = torch.nonzero(rep & (owner == o)).reshape(-1)  # ascending sample order
                r = r[torch.argsort(quarter[r], stable=True)]      # quarter-major (ABI 28)
                if r.numel() > cap:
                    raise RuntimeError(f"row-sharded exchange overflow: more than cap={cap} ids "
                                       "of one table for one owner in a batch; raise cap")
                slot_u[inv[r]] = torch.arange(r.numel())
                send[o, c, f * cap:f * cap + r.numel()] = (t[r] // W).to(torch.int32)
                send[o, c, F * cap + f] = r.numel()
            pos[f, s0:s0 + n] = (((owner * C + c) * F + f) * cap + slot_u[inv]).to(torch.int32)
        for o in range(W):
            if int(send[o, c, F * cap:].sum()) > bank.cap_rows:
                raise RuntimeError(f"row-sharded exchange overflow: more than cap_rows="
                                   f"{bank.cap_rows} distinct ids for one owner in a batch")
    return send.reshape(W, C * bank.part), pos


def _cpu_slots(bank: ShardedEmbeddingBank, recv: torch.Tensor, compact: bool) -> torch.Tensor:
    """The slot ids of a received ids message ([parts, F * cap]): the compact message
    carries the counts behind each part (and W * chunks parts)."""
    if compact:
        return recv.reshape(-1, bank.part)[:, :bank.n_tables * bank.cap]
    return recv


def _cpu_owner_rows(bank: ShardedEmbeddingBank, recv: torch.Tensor) -> torch.Tensor:
    F, cap = bank.n_tables, bank.cap
    flat = recv.reshape(-1).long()
    f_of = (torch.arange(flat.numel()) // cap) % F
    offs = torch.tensor(bank.row_offset, dtype=torch.long)[f_of]
    valid = flat >= 0
    rows = torch.zeros(flat.numel(), bank.row_stride, dtype=bank.weight.dtype)
    rows[valid] = bank.weight.detach()[offs[valid] + flat[valid]]
    return rows, offs, valid


class _CpuExchangeRowsFn(torch.autograd.Function):
    """forward: owner rows -> all_to_all -> rows at the sender's slots;
    backward: slot gradients -> reverse all_to_all -> owner SGD (lr / W)."""

    @staticmethod
    def forward(ctx, trigger, bank: ShardedEmbeddingBank, recv):
        # (recv: the slot ids, [parts, F * cap], _cpu_slots)
        rows, offs, valid = _cpu_owner_rows(bank, recv)
        ctx.bank, ctx.recv, ctx.offs, ctx.valid = bank, recv, offs, valid
        return bank.comm.exchange(rows.float())

    @staticmethod
    def backward(ctx, g):
        bank = ctx.bank
        g_recv = bank.comm.exchange(g.contiguous())
        flat = ctx.recv.reshape(-1).long()
        idx = (ctx.offs + flat)[ctx.valid]
        cols = bank.dim + (1 if bank.has_w else 0)
        upd = g_recv[ctx.valid][:, :cols].to(bank.weight.dtype)
        with torch.no_grad():
            w = bank.weight
            acc = torch.zeros(w.shape[0], cols, dtype=torch.float32)
            acc.index_add_(0, idx, upd.float())  # fixed (slot) order
            touched = torch.zeros(w.shape[0], dtype=torch.bool)
            touched[idx] = True
            lr = bank.current_lr() / bank.world
            w[touched, :cols] = (w[touched, :cols].float() - lr * acc[touched]).to(w.dtype)
        return None, None, None


def cpu_sharded_interact(bank: ShardedEmbeddingBank, ids, dense, dense_w, bias, use_fm2: bool,
                         first_order: bool, x0_cols: int, x0_dtype):
    from pytorchrec_amd import cpu_path
    B = ids[0].shape[0]
    compact = bank.use_compact(B)
    send, pos = cpu_bucketize_dedup(bank, ids) if compact else cpu_bucketize(bank, ids)
    recv = _cpu_slots(bank, bank.comm.exchange(send), compact)
    trig = torch.zeros(0, requires_grad=True) if torch.is_grad_enabled() else None
    rows = _CpuExchangeRowsFn.apply(trig, bank, recv)
    g = [rows.index_select(0, pos[f].long()) for f in range(bank.n_tables)]
    return cpu_path.interact_rows(g, bank.dim, dense, dense_w, bias, use_fm2, first_order,
                                  x0_cols, x0_dtype)


def sharded_interact(bank: ShardedEmbeddingBank, ids, dense, dense_w, bias, fm2: bool,
                     first_order: bool, x0_cols: int, x0_dtype):
    if not bank.weight.is_cuda:
        return cpu_sharded_interact(bank, ids, dense, dense_w, bias, fm2, first_order, x0_cols,
                                    x0_dtype)
    trigger = _trigger(bank)
    compact = bank.use_compact(ids[0].shape[0])
    if not compact:
        bank.check_slot_batch(ids[0].shape[0])
    fn = _CompactInteractFn if compact else _ShardedInteractFn
    return fn.apply(dense_w, bias, trigger, bank, ids, dense, fm2, first_order, int(x0_cols),
                    x0_dtype)


__all__ = ["ShardComm", "ShardedEmbeddingBank", "sharded_tables", "make_bank", "default_cap",
           "default_cap_rows", "sharded_interact", "shard_bucketize", "shard_gather",
           "shard_lookup_grad", "shard_bucketize_dedup", "shard_gather_wire", "shard_wire_unpack",
           "shard_wire_pack", "sender_plan_job", "sender_grad_sums", "owner_plan",
           "owner_plan_job", "owner_apply", "remote_desc", "shard_interact", "cpu_bucketize",
           "cpu_bucketize_dedup", "dedup_quarter"]
