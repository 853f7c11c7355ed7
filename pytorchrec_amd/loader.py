"""Columnar batch feed with pipelined host-to-device copies.

Reference behaviour replaced: ``SimpleDataReader.__getitem__`` returns
``dict(df.iloc[i])`` per SAMPLE (SimpleDataReader.py:323-331), ``IModel.fit``
collates the sample dicts with a ``DataLoader`` + ``default_collate``
(IModel.py:183-190), and ``train_step`` moves every tensor with its own blocking
``.to(device)`` (IModel.py:119).  At B=4096 that is ~4096 Python dicts and ~40
small synchronous copies per batch — the host becomes the bottleneck long before
a 127 µs GPU step does.

Here, once per epoch, the (shuffled) dataset is packed batch-major into ONE
pinned host buffer: batch j is a contiguous ``slot_bytes`` record holding every
column of its samples (``PackedLayout``: one 256-B aligned segment per column,
ids first).  A batch then crosses PCIe as ONE copy (655 KB at Criteo shape)
into one of ``depth`` device slots, enqueued ``depth - 1`` batches ahead on the
consumer's stream, so stream order alone keeps a slot from being refilled before
its step ran.  The copy is a libmrec kernel reading the pinned record over PCIe
(``mrec_batch_stage``, ``copy="kernel"``): with ``hipMemcpyAsync`` (a DMA
engine, ``copy="dma"``) or a side copy stream ordered by events
(``copy="side"``) a HIP graph launched behind the copy waits on the host
(measured 0.19-0.43 ms/step against 0.13 with resident batches,
``tools/h2d_probe.py``).  The
yielded batch dict holds views into the slot: the keys and per-sample meaning
are the reference's (``const.py:78-98``), plus ``"__dense__"`` = the dense
feature columns pre-stacked ``[n, k]`` in the order ``dense_group`` names them
(what ``DeepFM._dense`` reads, no ``torch.stack``).

Shuffling is a seeded permutation per epoch (``seed + epoch``), applied while
packing (one ``index_select`` per column).  ``prepare_epoch()`` packs the next
epoch ahead of time (e.g. outside a timed region).  On a CPU device batches are
views of the packed host buffer (no copy, config C1).

A yielded GPU batch is valid until ``depth - 1`` further batches have been
requested (its slot is then refilled); ``clone()`` what must outlive that.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, Iterator, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

from pytorchrec_amd import _mrec

_ALIGN = 256


def _as_tensor(x) -> Tensor:
    t = x if isinstance(x, Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if t.is_cuda:
        raise ValueError("ColumnarDataset columns live in host memory")
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    if not t.is_floating_point() and t.dtype != torch.uint8:
        # ids / lengths: int32 when every value fits (libmrec reads int32 in place)
        if t.numel() == 0 or (int(t.min()) >= -(1 << 31) and int(t.max()) < (1 << 31)):
            t = t.to(torch.int32)
        else:
            t = t.to(torch.int64)
    elif t.is_floating_point() and t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t.contiguous()


class ColumnarDataset(torch.utils.data.Dataset):
    """Equal-length host columns keyed by the reference's batch-dict names.

    ``columns``: name -> array of shape ``[N]`` or ``[N, ...]`` (numpy or CPU
    tensor).  Integer columns become int32 when their values fit (else int64),
    floats become fp32.  ``dense_group``: float ``[N]`` columns stacked once into
    ``"__dense__"`` ``[N, k]`` (the model's dense-column order).  Indexing
    returns the reference's per-sample dict (SimpleDataReader.py:323-331), so a
    plain ``DataLoader`` still works; ``ColumnarLoader`` is the fast path."""

    def __init__(self, columns: Mapping[str, object], dense_group: Optional[Sequence[str]] = None):
        cols = {str(k): _as_tensor(v) for k, v in columns.items()}
        if not cols:
            raise ValueError("ColumnarDataset needs at least one column")
        lens = {k: (v.shape[0] if v.dim() else -1) for k, v in cols.items()}
        n = next(iter(lens.values()))
        if any(v != n for v in lens.values()) or n < 0:
            raise ValueError(f"columns must share their first dimension: {lens}")
        self.n = int(n)
        self.dense_group = [str(k) for k in (dense_group or [])]
        for k in self.dense_group:
            if k not in cols or cols[k].dim() != 1 or cols[k].dtype != torch.float32:
                raise ValueError(f"dense_group column {k!r} must be a float [N] column")
        self.columns: Dict[str, Tensor] = {k: v for k, v in cols.items()
                                           if k not in self.dense_group}
        self.dense = (torch.stack([cols[k] for k in self.dense_group], dim=1).contiguous()
                      if self.dense_group else None)

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i) -> Dict[str, Tensor]:
        out = {k: v[i] for k, v in self.columns.items()}
        for j, k in enumerate(self.dense_group):
            out[k] = self.dense[i, j]
        return out

    def sources(self) -> List[Tuple[str, Tensor]]:
        """(segment name, [N, ...] tensor) in packing order: integer [N] columns
        (the ids) first, then the rest, then the stacked dense block."""
        items = sorted(self.columns.items(),
                       key=lambda kv: bool(kv[1].is_floating_point() or kv[1].dim() != 1))
        if self.dense is not None:
            items.append(("__dense__", self.dense))
        return items


class PackedLayout:
    """Byte layout of one batch record: per column a 256-B aligned segment
    ``[batch, *trailing]`` of the column's dtype.

    ``narrow`` (a kernel-copied GPU loader, ABI 29): the leading int32 ``[N]`` columns
    whose values all lie in [0, 65536) -- the ids of tables up to 65,536 rows -- are
    packed as 16-bit values in the HOST record and widened back to int32 by the copy
    into the device slot (``mrec_feed_job.widen_bytes``): a third less PCIe per C2
    batch.  Such a column's device segment is twice its host segment, so the widened
    prefix maps 1:2 and everything after it lands ``widen_bytes`` further on.
    ``record_bytes``: the host record; ``slot_bytes``: the device slot (the batch
    dict's views)."""

    def __init__(self, dataset: ColumnarDataset, batch: int, narrow: bool = False):
        self.batch = int(batch)
        self.dense_group = list(dataset.dense_group)
        # (name, dtype, trailing shape, device byte offset, bytes per sample, narrow)
        self.segments = []
        off = 0
        self.widen_bytes = 0
        prefix = bool(narrow)
        for name, t in dataset.sources():
            per = t.element_size() * int(math.prod(t.shape[1:]))
            nar = (prefix and t.dtype == torch.int32 and t.dim() == 1 and t.numel() > 0
                   and int(t.min()) >= 0 and int(t.max()) < 65536)
            prefix = nar  # only a leading run of columns is widened
            self.segments.append((name, t.dtype, tuple(t.shape[1:]), off, per, nar))
            if nar:
                hseg = (2 * self.batch + _ALIGN - 1) // _ALIGN * _ALIGN
                self.widen_bytes += hseg
                off += 2 * hseg
            else:
                off += (per * self.batch + _ALIGN - 1) // _ALIGN * _ALIGN
        self.slot_bytes = max(off, _ALIGN)
        self.record_bytes = max(off - self.widen_bytes, _ALIGN)

    def views(self, record: Tensor, n: int) -> Dict[str, Tensor]:
        """The batch dict over one DEVICE slot (uint8 ``[slot_bytes]``), first n
        samples (without narrow columns a host record is the same layout)."""
        out = {}
        for name, dt, trail, off, per, _ in self.segments:
            out[name] = record[off:off + per * self.batch].view(dt).view(self.batch, *trail)[:n]
        if "__dense__" in out:
            d = out["__dense__"]
            for j, k in enumerate(self.dense_group):
                out[k] = d[:, j]
        return out

    def pack(self, dataset: ColumnarDataset, order: Optional[Tensor], out: Tensor, n_batches: int):
        """Write the dataset (rows in ``order``, or in storage order) batch-major into
        ``out`` (uint8 ``[>= n_batches, record_bytes]``).  Bytes past the dataset's
        end in the last record are left as they are (views cut at n)."""
        N, B = dataset.n, self.batch
        full, rem = divmod(min(N, n_batches * B), B)
        srcs = dict(dataset.sources())
        for name, dt, trail, off, per, nar in self.segments:
            src = srcs[name]
            if order is not None:
                src = src.index_select(0, order)
            if nar:  # 16-bit in the host record (the uint16 bit pattern as int16)
                off, per, dt = off // 2, 2, torch.int16
                src = torch.where(src >= 32768, src - 65536, src).to(torch.int16)
            elif self.widen_bytes:
                off -= self.widen_bytes
            dst = out[:n_batches, off:off + per * B].view(dt).view(n_batches, B, *trail)
            if full:
                dst[:full].copy_(src[:full * B].view(full, B, *trail))
            if rem and full < n_batches:
                dst[full, :rem].copy_(src[full * B:full * B + rem])


class ColumnarLoader:
    """Iterates batch dicts of a ``ColumnarDataset`` on ``device`` (module doc).

    Mirrors the ``DataLoader`` arguments ``IModel.fit`` passes (batch_size,
    shuffle, drop_last; IModel.py:183-190).  ``depth`` device slots (>= 2) bound
        how far the copies run ahead; ``copy`` selects the H2D mechanism (module doc).
    A GPU batch of a ``copy="kernel"`` loader needs libmrec (raises
    ``MrecUnavailable`` without it: there is no silent fallback)."""

    def __init__(self, dataset: ColumnarDataset, batch_size: int, device=None,
                 shuffle: bool = False, drop_last: bool = False, seed: int = 0, depth: int = 3,
                 copy: str = "kernel"):
        if not isinstance(dataset, ColumnarDataset):
            raise TypeError("ColumnarLoader needs a ColumnarDataset")
        if int(batch_size) < 1:
            raise ValueError(f"batch_size must be >= 1, got {batch_size}")
        if int(depth) < 2:
            raise ValueError("depth must be >= 2")
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        self.seed = int(seed)
        self.depth = int(depth)
        if copy not in ("kernel", "dma", "side"):
            raise ValueError(f"copy must be 'kernel', 'dma' or 'side', got {copy!r}")
        self.copy = copy
        self.side_stream = copy == "side"
        self.epoch = 0
        # 16-bit ids in the host records when the copy is a kernel that widens them
        narrow = (self.device.type == "cuda" and copy == "kernel"
                  and os.environ.get("MREC_FEED_NARROW", "1") != "0")
        self.layout = PackedLayout(dataset, self.batch_size, narrow=narrow)
        self._host: Optional[Tensor] = None
        self._packed: Optional[List[int]] = None  # batch sizes of a prepared epoch
        self._slots: Optional[Tensor] = None
        self._copy_stream = None
        self._copied: List = []
        self._released: List = []
        self._reading = None  # event after the latest enqueued read of the host buffer
        self._iterating = False

    def __len__(self) -> int:
        n, b = self.dataset.n, self.batch_size
        return n // b if self.drop_last else -(-n // b)

    def _sizes(self) -> List[int]:
        n, b = self.dataset.n, self.batch_size
        return [min(b, n - j * b) for j in range(len(self))]

    def _order(self) -> Optional[Tensor]:
        if not self.shuffle:
            return None
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        return torch.randperm(self.dataset.n, generator=g)

    def prepare_epoch(self) -> List[int]:
        """Pack the next epoch into the host buffer (once; the next iteration uses it).
        Not while an epoch is being iterated: its remaining batches are staged from
        this same buffer (RuntimeError).  Before packing it waits for the device
        copies already enqueued from the buffer (the last batches of the previous
        epoch may still be queued behind the steps)."""
        if self._iterating:
            raise RuntimeError("ColumnarLoader.prepare_epoch() while an epoch is being "
                               "iterated: finish (or close) that iteration first")
        if self._packed is None:
            sizes = self._sizes()
            nb = max(len(sizes), 1)
            if self._reading is not None:
                self._reading.synchronize()  # enqueued copies of the last epoch read the buffer
            if self._host is None or self._host.shape[0] < nb:
                self._host = torch.empty(nb, self.layout.record_bytes, dtype=torch.uint8,
                                         pin_memory=self.device.type == "cuda")
            self.layout.pack(self.dataset, self._order(), self._host, nb)
            self.epoch += 1
            self._packed = sizes
        return self._packed

    def _take_epoch(self) -> List[int]:
        sizes = self.prepare_epoch()
        self._packed = None
        return sizes

    def _ensure_slots(self):
        if self._slots is None:
            dev = self.device
            self._slots = torch.empty(self.depth, self.layout.slot_bytes, dtype=torch.uint8,
                                      device=dev)
            self._copy_stream = torch.cuda.Stream(device=dev)
            self._copied = [torch.cuda.Event() for _ in range(self.depth)]
            self._released = [torch.cuda.Event() for _ in range(self.depth)]

    def slot_views(self, slot: int, n: Optional[int] = None) -> Dict[str, Tensor]:
        """Batch dict over device slot ``slot`` (e.g. to capture a HIP graph per slot)."""
        self._ensure_slots()
        return self.layout.views(self._slots[slot], self.batch_size if n is None else n)

    def iter_slots(self) -> Iterator[Tuple[int, int]]:
        """GPU pipeline: yields (slot, n) once the batch's copy is ordered before
        the current stream's next work; the caller enqueues its work on
        ``slot_views(slot, n)`` (or replays a graph captured over them) before
        asking for the next batch."""
        if self.device.type != "cuda":
            raise RuntimeError("iter_slots needs a cuda device")
        self._ensure_slots()
        sizes = self._take_epoch()
        cs, host = self._copy_stream, self._host
        if self._reading is None:
            self._reading = torch.cuda.Event()
        self._iterating = True
        try:
            issued = 0
            for i, n in enumerate(sizes):
                while issued < min(len(sizes), i + self.depth):
                    s = issued % self.depth
                    if self.copy == "kernel":  # stream order alone protects the slot
                        _mrec.call("mrec_batch_stage_ex", self._slots[s].data_ptr(),
                                   host[issued].data_ptr(), self.layout.record_bytes,
                                   self.layout.widen_bytes, _mrec.stream_handle(self.device))
                        self._reading.record(torch.cuda.current_stream(self.device))
                    elif self.copy == "dma":
                        self._slots[s].copy_(host[issued], non_blocking=True)
                        self._reading.record(torch.cuda.current_stream(self.device))
                    else:
                        with torch.cuda.stream(cs):
                            cs.wait_event(self._released[s])  # the consumer's last use of slot s
                            self._slots[s].copy_(host[issued], non_blocking=True)
                            self._copied[s].record(cs)
                            self._reading.record(cs)
                    issued += 1
                s = i % self.depth
                if self.side_stream:
                    torch.cuda.current_stream(self.device).wait_event(self._copied[s])
                yield s, n
                if self.side_stream:
                    self._released[s].record(torch.cuda.current_stream(self.device))
        finally:
            self._iterating = False

    # -- graph-captured steps, the H2D copy inside the step (ABI 27) ---------------
    def capture_steps(self, step) -> "GraphEpoch":
        """Capture ONE HIP graph of ``depth`` train steps ``step(batch_dict)``: step j
        reads device slot j while the record ``depth - 1`` batches ahead is copied into
        the slot step j - 1 read (``mrec_feed_job``: the record index is a device
        cursor, so every replay stages the next records with no host work).  The copy
        runs in extra workgroups of the step's fused-tower weight-gradient launch
        (``mrec_tower_dw_ex``: PCIe reads beside L2-bound tiles; a graph branch on a
        side stream was serialised by the graph executor), or after the step when the
        model has none (``mrec_batch_stage_cursor``).  Call ``step`` eagerly on
        ``slot_views`` first (warm-up).  Epochs are then run by
        ``GraphEpoch.replays()``; they need full batches in a multiple of ``depth``."""
        if self.device.type != "cuda" or self.copy != "kernel":
            raise RuntimeError("capture_steps needs a cuda device and copy='kernel'")
        from pytorchrec_amd import dense as dense_ops
        self.prepare_epoch()  # the pinned epoch buffer the graph reads (fixed address)
        self._ensure_slots()
        state = torch.zeros(2, dtype=torch.int64, device=self.device)
        g = torch.cuda.CUDAGraph()
        host = self._host
        jobs = [_mrec.FeedJob(self._slots[(j + self.depth - 1) % self.depth].data_ptr(),
                              host.data_ptr(), self.layout.record_bytes, host.shape[0],
                              state.data_ptr(), self.layout.widen_bytes)
                for j in range(self.depth)]
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for j in range(self.depth):
                    dense_ops.set_feed_job(jobs[j])
                    step(self.layout.views(self._slots[j], self.batch_size))
                    left = dense_ops.take_feed_job()
                    if left is not None:  # no tower weight-gradient launch in this step
                        _mrec.call("mrec_batch_stage_job", ctypes.byref(left),
                                   _mrec.stream_handle(self.device))
        finally:
            # a step that raised mid-capture leaves its job set: the next eager
            # tower_dw would take it and copy through this (freed) cursor
            dense_ops.take_feed_job()
        return GraphEpoch(self, g, state, host, jobs)

    def __iter__(self) -> Iterator[Dict[str, Tensor]]:
        if self.device.type == "cuda":
            for s, n in self.iter_slots():
                yield self.layout.views(self._slots[s], n)
        else:
            sizes = self._take_epoch()
            self._iterating = True  # the batches are views of the host buffer
            try:
                for j, n in enumerate(sizes):
                    yield self.layout.views(self._host[j], n)
            finally:
                self._iterating = False


class GraphEpoch:
    """Epochs of a ``ColumnarLoader`` run by replaying the graph ``capture_steps``
    captured (``depth`` steps per replay)."""

    def __init__(self, loader: ColumnarLoader, graph, state: Tensor, host: Tensor, jobs):
        self.loader, self.graph, self.state, self.host = loader, graph, state, host
        self.jobs = jobs  # (the captured kernels' argument blocks point at these buffers)

    def replays(self) -> Iterator[int]:
        """Run one epoch: stage its first ``depth - 1`` batches, then replay the
        graph len / depth times (yielding the first batch index of each replay)."""
        ld = self.loader
        sizes = ld._take_epoch()
        d = ld.depth
        if ld._host.data_ptr() != self.host.data_ptr():
            raise RuntimeError("the loader's host buffer moved since capture_steps")
        if any(n != ld.batch_size for n in sizes) or len(sizes) % d:
            raise ValueError(f"graph epochs need full batches in a multiple of depth={d} "
                             f"(got {len(sizes)} batches)")
        ld._iterating = True
        try:
            for j in range(min(d - 1, len(sizes))):
                _mrec.call("mrec_batch_stage_ex", ld._slots[j].data_ptr(), ld._host[j].data_ptr(),
                           ld.layout.record_bytes, ld.layout.widen_bytes,
                           _mrec.stream_handle(ld.device))
            self.state.zero_()
            self.state[0] = d - 1
            for r in range(len(sizes) // d):
                self.graph.replay()
                yield r * d
            if ld._reading is None:
                ld._reading = torch.cuda.Event()
            ld._reading.record(torch.cuda.current_stream(ld.device))
        finally:
            ld._iterating = False
