"""Embedding bank: F categorical tables packed for the MI355X hot path.

``EmbeddingBank`` replaces the F ``torch.nn.Embedding`` tables (plus the
``Embedding(rows, 1)`` first-order biases) that a reference model builds in
``IModel._init_weights`` (torchrec/model/FunkSVD.py:39-41, SVDPP.py:36-42).  All
tables live in ONE parameter ``weight`` of shape [total_rows, row_stride]:

    row r of table f  ->  weight[row_offset[f] + r] = [ v(dim) | w | pad ]

with the row padded to a power-of-two byte width (64 B for bf16 dim 16 + w) so
each lookup is one aligned, coalesced request (DESIGN.md §Data layout).

The autograd functions here are the only way the models touch the tables on a
GPU: they call libmrec (``_mrec``) and raise if it is missing.  On a CPU device
(config C1, the reference's own CPU path) the same math runs as plain torch
index_select / index_add (``cpu_path``) — an explicit device dispatch, never a
fallback for a GPU tensor.

Update modes (``EmbeddingBank.update``):
  "dense"     backward materialises the dense table gradient exactly like
              ``aten::embedding_dense_backward`` so any torch optimizer works
              (reference semantics, IModel.py:120-124);
  "sgd"       the backward applies row-sparse SGD in place (identical to dense
              SGD without momentum / weight decay), the gradient never exists;
              ``IModel.compile`` switches to it when the compiled optimizer is
              plain SGD (SURVEY.md §7 hard part 5);
  "adagrad" / "rowwise_adagrad" / "adam"
              the same with a fused optimizer whose state lives beside the bank
              (include/mrec.h MREC_BWD_ADAGRAD / _ROWWISE_ADAGRAD / _ADAM):
              torch.optim.Adagrad, row-wise Adagrad (``optim.RowWiseAdagrad``),
              and dense-compatible Adam / the reference AdamW (rows catch up on the
              zero-gradient steps they missed; ``flush_optimizer`` brings every row
              to the current step).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import torch

from pytorchrec_amd import _mrec, cpu_path


def _row_stride(dim: int, has_w: bool, dtype: torch.dtype) -> int:
    es = torch.tensor([], dtype=dtype).element_size()
    need = (dim + (1 if has_w else 0)) * es
    b = 16
    while b < need:
        b *= 2
    if b > 256:
        raise ValueError(f"row of {need} bytes exceeds 256 B (dim too large for one bank row)")
    return b // es


class EmbeddingBank(torch.nn.Module):
    """F embedding tables (+ optional first-order weight column) in one tensor.

    ``category_nums[f]`` rows for table f (``CategoricalColumn.category_num``,
    CategoricalColumn.py:9-14).  ``weight`` is initialised by the host model's
    ``IModel._reset_weights`` (normal(0, 0.01), IModel.py:61-68): the class name
    contains "Embedding" so the reference's type-name match applies to it.
    """

    def __init__(self, category_nums: Sequence[int], dim: int, with_first_order: bool = False,
                 dtype: torch.dtype = torch.float32, update: str = "dense", device=None):
        super().__init__()
        if len(category_nums) < 1:
            raise ValueError("need at least one table")
        if update not in ("dense", "sgd"):
            raise ValueError(f"update must be 'dense' or 'sgd', got {update!r}")  # (others: use_fused_optimizer)
        es = torch.tensor([], dtype=dtype).element_size()
        if dim <= 0 or (dim * es) % 16:
            raise ValueError(f"dim*{es}B must be a positive multiple of 16 bytes (dim={dim})")
        self.category_nums = [int(n) for n in category_nums]
        self.dim = int(dim)
        self.has_w = bool(with_first_order)
        self.row_stride = _row_stride(self.dim, self.has_w, dtype)
        offs, acc = [], 0
        for n in self.category_nums:
            offs.append(acc)
            acc += n
        self.row_offset = offs
        self.total_rows = acc
        # zeros: the pad columns past [v | w] stay zero (never read by a kernel, but
        # they travel into state_dict / checkpoints, so no uninitialised bits)
        self.weight = torch.nn.Parameter(
            torch.zeros(acc, self.row_stride, dtype=dtype, device=device),
            requires_grad=(update == "dense"))
        self.update = update
        self.sgd_lr: Optional[float] = None
        self.sgd_group = None  # optimizer param group the fused SGD lr is read from
        self.stochastic_rounding = dtype == torch.bfloat16
        self.check_ids = True  # raise IndexError on out-of-range ids (syncs once per call)
        self._seed = 0x5eed
        self._desc = None
        self._optim = None  # _mrec.Optim of a fused optimizer (use_fused_optimizer)
        self.optim_state = None
        self._step = None  # device uint64 counter (SR bits stay fresh under graph replay)

    @property
    def n_tables(self) -> int:
        return len(self.category_nums)

    # -- optimizer integration -------------------------------------------------
    def use_fused_sgd(self, lr: float, group=None):
        self.update = "sgd"
        self.sgd_lr = float(lr)
        self.sgd_group = group
        self.weight.requires_grad_(False)
        self._set_optim(None)

    def use_dense_grad(self):
        self.update = "dense"
        self.weight.requires_grad_(True)
        self._set_optim(None)

    FUSED_OPTIMIZERS = ("adagrad", "rowwise_adagrad", "adam")

    def use_fused_optimizer(self, kind: str, group, *, eps: float, betas=(0.9, 0.999),
                            weight_decay: float = 0.0, decoupled: bool = False,
                            bias_correction: bool = True, grad_scale: float = 1.0):
        """Row-sparse fused optimizer: the state tensors are allocated here (zeros,
        as the dense optimizers start), ``group`` supplies the lr each step."""
        if kind not in self.FUSED_OPTIMIZERS:
            raise ValueError(f"fused optimizer must be one of {self.FUSED_OPTIMIZERS}")
        dev = self.weight.device
        f32 = dict(dtype=torch.float32, device=dev)
        ld = int(_mrec.lib().mrec_emb_optim_state_ld(self.dim, int(self.has_w)))
        st = {}
        if kind == "adagrad":
            st["s0"] = torch.zeros(self.total_rows, ld, **f32)
        elif kind == "rowwise_adagrad":
            st["s0"] = torch.zeros(self.total_rows, 2, **f32)
        else:
            st["s0"] = torch.zeros(self.total_rows, ld, **f32)
            st["s1"] = torch.zeros(self.total_rows, ld, **f32)
            st["row_step"] = torch.zeros(self.total_rows, dtype=torch.int32, device=dev)
            st["t"] = torch.zeros(1, dtype=torch.int64, device=dev)
        flags = ((_mrec.OPT_DECOUPLED_WD if decoupled else 0)
                 | (0 if bias_correction else _mrec.OPT_NO_BIAS_CORRECTION))
        self.optim_state = st
        kind_code = {"adagrad": _mrec.BWD_ADAGRAD, "rowwise_adagrad": _mrec.BWD_ROWWISE_ADAGRAD,
                     "adam": _mrec.BWD_ADAM}[kind]
        self._optim = _mrec.Optim(kind_code, float(group["lr"]), float(betas[0]), float(betas[1]),
                                  float(eps),
                                  float(weight_decay), float(grad_scale), flags,
                                  st["s0"].data_ptr(), _mrec.ptr(st.get("s1")),
                                  _mrec.ptr(st.get("row_step")), _mrec.ptr(st.get("t")), ld)
        self.update = kind
        self.sgd_lr = None
        self.sgd_group = group
        self.weight.requires_grad_(False)
        self._set_optim(self._optim)

    def _set_optim(self, optim):
        self._optim = optim
        if optim is None:
            self.optim_state = None
        if self._desc is not None:
            self._desc.set_optim(optim)

    @property
    def fused(self) -> bool:
        """The update happens inside the backward (no table gradient exists)."""
        return self.update != "dense"

    def apply_mode(self):
        """(mrec_bwd_mode, lr) of this step's fused update; for Adam the device step
        counter advances first (stream-ordered: right under graph replay too)."""
        if self.update == "sgd":
            mode = (_mrec.BWD_SGD_SR if (self.stochastic_rounding and
                                         self.weight.dtype == torch.bfloat16) else _mrec.BWD_SGD)
            return mode, self.current_lr()
        if self.update == "dense":
            return _mrec.BWD_DENSE_GRAD, 0.0
        if self.update == "adam":
            new_lr = ctypes.c_float(self.current_lr()).value
            if new_lr != self._optim.lr and self.weight.is_cuda:
                # the lr changed (a scheduler, a manual decay): rows not looked up since
                # the last step owe their missed zero-gradient steps at the OLD lr, as
                # dense Adam took them; bring every row to the current step first
                _mrec.call("mrec_emb_optim_flush", self.desc().ref(), _mrec.BWD_ADAM,
                           float(self._optim.lr), _mrec.stream_handle())
            self.optim_state["t"].add_(1)
            self._optim.lr = new_lr  # catch-up lr of stale-row reads from now on
        mode = {"adagrad": _mrec.BWD_ADAGRAD, "rowwise_adagrad": _mrec.BWD_ROWWISE_ADAGRAD,
                "adam": _mrec.BWD_ADAM}[self.update]
        return mode, self.current_lr()

    def flush_optimizer(self):
        """Dense-compatible Adam: bring the rows not looked up at the current step
        up to it (their missed zero-gradient steps), so the table equals dense
        Adam's.  Other update modes: nothing to do."""
        if self.update == "adam" and self.weight.is_cuda:
            _mrec.call("mrec_emb_optim_flush", self.desc().ref(), _mrec.BWD_ADAM,
                       float(self.current_lr()), _mrec.stream_handle())

    def current_lr(self) -> float:
        if self.sgd_group is not None:
            return float(self.sgd_group["lr"])
        if self.sgd_lr is None:
            raise RuntimeError("fused SGD update without a learning rate")
        return self.sgd_lr

    def step_counter(self) -> torch.Tensor:
        if self._step is None or self._step.device != self.weight.device:
            self._step = torch.zeros(1, dtype=torch.int64, device=self.weight.device)
        return self._step

    def next_seed(self) -> int:
        self._seed = (self._seed * 6364136223846793005 + 1442695040888963407) & (2 ** 64 - 1)
        return self._seed

    @torch.no_grad()
    def zero_pad_(self):
        """Zero the row-pitch pad columns (after an init that wrote whole rows)."""
        used = self.dim + (1 if self.has_w else 0)
        if used < self.row_stride:
            self.weight[:, used:].zero_()
        return self

    def check_flags(self):
        """Raise if a large-batch backward since the last check could not finish its
        huge-segment phases (the workspace's sticky error word, ABI 25: those rows were
        left un-updated, never updated from partial sums).  Syncs once; clears the
        word.  IModel.fit calls it at the end of every epoch, the id-checking mode
        after every large backward."""
        cache = getattr(self, "_large_ws_cache", None)
        if cache is None:
            return
        off = int(_mrec.lib().mrec_emb_bwd_large_error_offset())
        word = cache[1][off:off + 4].view(torch.int32)
        err = int(word.item())
        if err:
            word.zero_()
            if err == 2:
                raise RuntimeError("embedding backward: a bucket of the large-batch plan held "
                                   "more distinct rows than its LDS hash (a bank of more than "
                                   "2^24 rows); some rows of that step were not updated")
            raise RuntimeError("embedding backward: the huge-segment phases of a large-batch "
                               "update timed out waiting for each other (a stalled GPU); the "
                               "rows hit > 2048 times in that step were not updated")

    # -- table views (for checkpoints / tests) ----------------------------------
    def table(self, f: int) -> torch.Tensor:
        o = self.row_offset[f]
        return self.weight[o:o + self.category_nums[f], :self.dim]

    def first_order(self, f: int) -> torch.Tensor:
        if not self.has_w:
            raise ValueError("bank has no first-order column")
        o = self.row_offset[f]
        return self.weight[o:o + self.category_nums[f], self.dim]

    def desc(self) -> _mrec.BankDesc:
        if self._desc is None or self._desc.weight is not self.weight:
            self._desc = _mrec.BankDesc(self.weight, self.row_offset, self.category_nums,
                                        self.dim, self.has_w)
            self._desc.set_optim(self._optim)
        return self._desc

    def extra_repr(self) -> str:
        return (f"tables={self.n_tables}, rows={self.total_rows}, dim={self.dim}, "
                f"first_order={self.has_w}, row_stride={self.row_stride}, "
                f"dtype={self.weight.dtype}, update={self.update}")


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------


def _oob_flag(bank: EmbeddingBank, device) -> Optional[torch.Tensor]:
    return torch.zeros(1, dtype=torch.int32, device=device) if bank.check_ids else None


def _raise_if_oob(flag: Optional[torch.Tensor]):
    if flag is not None and int(flag.item()) != 0:
        raise IndexError("index out of range in self")


class PaddedIds(list):
    """Per-field id tensors whose negative ids are padding slots (mrec_ids.pad_negative):
    the gather returns a zero row for them and the backward skips them."""
    pad_negative = True


def _ids_desc(ids: Sequence[torch.Tensor], start: int = 0, count: Optional[int] = None):
    pn = getattr(ids, "pad_negative", False)
    if start == 0 and count is None:
        return _mrec.IdsDesc(ids, pad_negative=pn)
    return _mrec.IdsDesc([t[start:start + count] for t in ids], pad_negative=pn)


def _plan(bank: EmbeddingBank, ids, start: int, count: int, flag):
    n = bank.n_tables
    ws_bytes = _mrec.lib().mrec_emb_bwd_workspace_size(n, count)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=bank.weight.device)
    idd = _ids_desc(ids, start, count) if (start or count != ids[0].shape[0]) else _ids_desc(ids)
    _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), idd.ref(), count, ws.data_ptr(), ws_bytes,
               _mrec.ptr(flag), bank.step_counter().data_ptr(), _mrec.stream_handle())
    return ws, ws_bytes


_SIDE = {}


def _side_stream(device) -> torch.cuda.Stream:
    st = _SIDE.get(device)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _SIDE[device] = st
    return st


class _AsyncPlanBase:
    """A sorted-segment plan launched on a side stream: it depends only on the
    ids, so it runs concurrently with the interaction kernel and the MLP forward;
    the backward waits on its event before the apply kernel."""

    def __init__(self, device, launch, inputs):
        cur = torch.cuda.current_stream(device)
        side = _side_stream(device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self.ws, self.ws_bytes = launch()
            self.event = torch.cuda.Event()
            self.event.record(side)
        self.ws.record_stream(cur)
        for t in inputs:
            t.record_stream(side)

    def get(self):
        torch.cuda.current_stream(self.ws.device).wait_event(self.event)
        return self.ws, self.ws_bytes


class _AsyncPlan(_AsyncPlanBase):
    def __init__(self, bank: EmbeddingBank, ids, batch: int):
        super().__init__(bank.weight.device, lambda: _plan(bank, ids, 0, batch, None), ids)


def _make_plan(bank: EmbeddingBank, ids, batch: int):
    if torch.cuda.is_current_stream_capturing():
        # a HIP graph runs its kernels one after another anyway, and the side
        # stream's fork/join cost 11 us per step (C2): plan in the backward
        return None
    return _AsyncPlan(bank, ids, batch)


def _apply(bank: EmbeddingBank, ws, ws_bytes, count, dx=None, dfm=None, fm_sum=None, x0=None,
           dw=None, grad=None):
    """Run the fused backward for lookups [0, count) described by ``ws``; the
    per-sample tensors must already be sliced to the same chunk."""
    mode, lr = bank.apply_mode()
    dx_dt = _mrec.dtype_code(dx.dtype) if dx is not None else _mrec.F32
    x0_dt = _mrec.dtype_code(x0.dtype) if x0 is not None else _mrec.F32
    # deferred MLP weight-gradient reductions (+ fused SGD) ride along this launch
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    _mrec.call("mrec_emb_bwd_apply_ex", bank.desc().ref(), count, ws.data_ptr(), ws_bytes,
               _mrec.ptr(dx), dx_dt, dx.stride(0) if dx is not None else 0,
               _mrec.ptr(dfm), _mrec.ptr(fm_sum), _mrec.ptr(x0), x0_dt,
               x0.stride(0) if x0 is not None else 0, _mrec.ptr(dw), mode, float(lr),
               bank.next_seed(), bank.step_counter().data_ptr(), _mrec.ptr(grad), len(jobs),
               arr, _mrec.stream_handle())
    del jobs


def _chunks(batch: int):
    step = _mrec.BWD_MAX_BATCH
    return [(s, min(step, batch - s)) for s in range(0, batch, step)] or [(0, 0)]


LARGE_MAX_ROWS = 1 << 24  # banks up to this many rows take the large-batch path
# MREC_LARGE_BATCH=0: chunked plan/apply pairs instead (one SGD step per chunk)
LARGE_BATCH = os.environ.get("MREC_LARGE_BATCH", "1") == "1"
# MREC_LARGE_FUSED=0: the plan / apply pair instead of mrec_emb_bwd_large_fused
LARGE_FUSED = os.environ.get("MREC_LARGE_FUSED", "1") == "1"


def _large_ws(bank: EmbeddingBank, batch: int) -> torch.Tensor:
    """The large-batch workspace, kept on the bank per batch size: zeroed once at
    allocation, every mrec_emb_bwd_large_apply leaves its zero region zero."""
    cache = getattr(bank, "_large_ws_cache", None)
    if cache is None or cache[0] != batch or cache[1].device != bank.weight.device:
        if cache is not None and not torch.cuda.is_current_stream_capturing():
            bank.check_flags()  # an earlier step's sticky error word must not be dropped
        nbytes = _mrec.lib().mrec_emb_bwd_large_workspace_size(bank.desc().ref(), batch)
        cache = (batch, torch.zeros(nbytes, dtype=torch.uint8, device=bank.weight.device))
        bank._large_ws_cache = cache
    return cache[1]


def _backward_large(bank: EmbeddingBank, ids, batch, grad, dx=None, dfm=None, fm_sum=None,
                    x0=None, dw=None):
    """One device-wide plan + ONE update per row for batches beyond a plan
    workgroup (DIN's B x L history lookups): emb_bwd_large.hip, one call
    (mrec_emb_bwd_large_fused: the bucketed plan with the updates in the bucket
    kernel; the plan / apply pair when the batch is too large for it)."""
    ws = _large_ws(bank, batch)
    mode, lr = bank.apply_mode()
    if not LARGE_FUSED:
        _mrec.call("mrec_emb_bwd_large_plan", bank.desc().ref(), _ids_desc(ids).ref(), batch,
                   ws.data_ptr(), ws.numel(), None, _mrec.stream_handle())
        _mrec.call("mrec_emb_bwd_large_apply", bank.desc().ref(), batch, ws.data_ptr(),
                   ws.numel(), *_large_apply_args(bank, grad, dx, dfm, fm_sum, x0, dw, mode, lr))
        return
    # deferred MLP weight-gradient reductions (DIN's top tower) ride along the bucket kernel
    from pytorchrec_amd import dense as dense_ops
    jobs = dense_ops.take_pending(dense_ops.CO_REDUCE_MAX)
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs]) if jobs else None
    args = _large_apply_args(bank, grad, dx, dfm, fm_sum, x0, dw, mode, lr)
    _mrec.call("mrec_emb_bwd_large_fused_ex", bank.desc().ref(), _ids_desc(ids).ref(), batch,
               ws.data_ptr(), ws.numel(), None, *args[:-1], len(jobs), arr, args[-1])
    del jobs
    if bank.check_ids and not torch.cuda.is_current_stream_capturing():
        bank.check_flags()


def _large_apply_args(bank, grad, dx, dfm, fm_sum, x0, dw, mode, lr):
    """The apply arguments of mrec_emb_bwd_large_apply / _fused after the workspace."""
    return (_mrec.ptr(dx), _mrec.dtype_code(dx.dtype) if dx is not None else _mrec.F32,
            dx.stride(0) if dx is not None else 0, _mrec.ptr(dfm), _mrec.ptr(fm_sum),
            _mrec.ptr(x0), _mrec.dtype_code(x0.dtype) if x0 is not None else _mrec.F32,
            x0.stride(0) if x0 is not None else 0, _mrec.ptr(dw), mode, float(lr),
            bank.next_seed(), bank.step_counter().data_ptr(), _mrec.ptr(grad),
            _mrec.stream_handle())


def _backward_into_bank(bank: EmbeddingBank, ids, batch, plan_ws, dx=None, dfm=None,
                        fm_sum=None, x0=None, dw=None):
    """Shared backward: returns the dense grad (dense mode) or None (fused SGD)."""
    grad = None
    if bank.update == "dense":
        grad = torch.zeros_like(bank.weight)
    if plan_ws is not None:
        ws, wsb = plan_ws.get() if isinstance(plan_ws, _AsyncPlan) else plan_ws
        _apply(bank, ws, wsb, batch, dx, dfm, fm_sum, x0, dw, grad)
        return grad
    if batch > _mrec.BWD_MAX_BATCH and bank.total_rows <= LARGE_MAX_ROWS and LARGE_BATCH:
        _backward_large(bank, ids, batch, grad, dx, dfm, fm_sum, x0, dw)
        return grad
    if bank.update == "adam" and batch > _mrec.BWD_MAX_BATCH:
        raise NotImplementedError("fused Adam takes one apply per step: batches above "
                                  f"{_mrec.BWD_MAX_BATCH} lookups per table need the large-batch "
                                  "path (MREC_LARGE_BATCH=1, banks up to 2^24 rows)")
    for s, c in _chunks(batch):
        if c == 0:
            continue
        ws, wsb = _plan(bank, ids, s, c, None)
        sl = (lambda t: None if t is None else t[s:s + c])
        _apply(bank, ws, wsb, c, sl(dx), sl(dfm), sl(fm_sum), sl(x0), sl(dw), grad)
    return grad


def _needs_backward(bank: EmbeddingBank) -> bool:
    return torch.is_grad_enabled() and (bank.fused or bank.weight.requires_grad)


# ----------------------------------------------------------------------------
# autograd: plain multi-table gather  (nn.Embedding x F)
# ----------------------------------------------------------------------------


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, trigger, bank: EmbeddingBank, ids: List[torch.Tensor], out_dtype,
                want_w: bool, need_bwd: bool, din_src=None):
        B = ids[0].shape[0]
        F, D = bank.n_tables, bank.dim
        dev = weight.device
        out = torch.empty(B, F * D, dtype=out_dtype, device=dev)
        w_out = torch.empty(B, F, dtype=torch.float32, device=dev) if want_w else None
        flag = _oob_flag(bank, dev)
        if B and din_src is not None:  # DIN: the ids are built by the gather launch itself
            iid, cid, his, hcat = din_src
            _mrec.call("mrec_din_gather", bank.desc().ref(), iid.data_ptr(), cid.data_ptr(),
                       his.data_ptr(), his.stride(0), hcat.data_ptr(), hcat.stride(0),
                       _mrec.dtype_code(his.dtype), his.shape[0], his.shape[1],
                       ids[0].data_ptr(), ids[1].data_ptr(), out.data_ptr(),
                       _mrec.dtype_code(out_dtype), out.stride(0), _mrec.ptr(flag),
                       _mrec.stream_handle())
        elif B:
            _mrec.call("mrec_emb_gather_fwd", bank.desc().ref(), _ids_desc(ids).ref(), B,
                       out.data_ptr(), _mrec.dtype_code(out_dtype), out.stride(0),
                       _mrec.ptr(w_out), _mrec.ptr(flag), _mrec.stream_handle())
        plan_ws = None
        if need_bwd and 0 < B <= _mrec.BWD_MAX_BATCH:
            plan_ws = _make_plan(bank, ids, B)
        _raise_if_oob(flag)
        ctx.bank, ctx.ids, ctx.B, ctx.plan_ws = bank, ids, B, plan_ws
        if want_w:
            return out, w_out
        return out

    @staticmethod
    def backward(ctx, dout, dw_out=None):
        bank = ctx.bank
        dx = dout.contiguous() if dout is not None else None
        dw = None
        if dw_out is not None:
            if bank.n_tables != 1:
                raise NotImplementedError("first-order grads through gather need one table "
                                          "per call; use interact() for multi-field models")
            dw = dw_out.reshape(-1).contiguous().float()
        grad = _backward_into_bank(bank, ctx.ids, ctx.B, ctx.plan_ws, dx=dx, dw=dw)
        return grad, None, None, None, None, None, None, None


def gather(bank: EmbeddingBank, ids: Sequence[torch.Tensor], out_dtype=None, with_w=False,
           pad_negative: bool = False, din_src=None):
    """out[b, f*D:(f+1)*D] = table_f[ids[f][b]] — F ``nn.Embedding`` lookups.

    Returns [B, F*D] (and [B, F] first-order weights if ``with_w``).  With
    ``pad_negative`` a negative id is a padding slot: a zero row, no gradient.
    ``din_src`` = (iid, cid, his, hcat): ``ids`` are int32 output buffers that the
    launch fills with DIN's padded lookup ids (mrec_din_gather; GPU only).
    """
    ids = PaddedIds(ids) if pad_negative else list(ids)
    if len(ids) != bank.n_tables:
        raise ValueError(f"expected {bank.n_tables} id tensors, got {len(ids)}")
    out_dtype = out_dtype or bank.weight.dtype
    if not bank.weight.is_cuda:
        return cpu_path.gather(bank, ids, out_dtype, with_w)
    trigger = _trigger(bank)
    # (grad mode is off inside Function.forward: decide here whether a backward
    # will run, so the plan can be queued ahead of it)
    return _GatherFn.apply(bank.weight, trigger, bank, ids, out_dtype, with_w,
                           _needs_backward(bank), din_src)


_TRIGGERS = {}


def _trigger(bank: EmbeddingBank):
    """A 0-element leaf that requires grad, so autograd calls our backward even when
    the bank itself is updated in place (fused SGD, weight.requires_grad False)."""
    if not bank.fused or not torch.is_grad_enabled():
        return None
    t = _TRIGGERS.get(bank.weight.device)
    if t is None:
        t = torch.zeros(0, device=bank.weight.device, requires_grad=True)
        _TRIGGERS[bank.weight.device] = t
    return t


# ----------------------------------------------------------------------------
# autograd: fused gather + FM2 + first order + deep-input builder
# ----------------------------------------------------------------------------


class _InteractFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, dense_w, bias, trigger, bank: EmbeddingBank, ids, dense, fm2: bool,
                first_order: bool, x0_cols: int, x0_dtype, need_bwd: bool):
        B = ids[0].shape[0]
        dev = weight.device
        n_dense = 0 if dense is None else dense.shape[1]
        flags = (_mrec.INTERACT_FM2 if fm2 else 0) | (_mrec.INTERACT_FIRST_ORDER if first_order else 0)
        x0 = None
        ret_x0 = bool(x0_cols)
        if fm2 and need_bwd and not x0_cols:
            # the FM gradient of lookup (b, f) is dfm_b * (fm_sum_b - v_bf): keep the
            # gathered rows for the backward (an exact copy in the bank's dtype)
            x0_cols = (bank.n_tables * bank.dim + n_dense + 7) // 8 * 8
            x0_dtype = weight.dtype
        if x0_cols:
            x0 = torch.empty(B, x0_cols, dtype=x0_dtype, device=dev)
        logit = torch.empty(B, dtype=torch.float32, device=dev)
        fm_sum = torch.empty(B, bank.dim, dtype=torch.float32, device=dev) if fm2 else None
        flag = _oob_flag(bank, dev)
        plan_ws, job = None, None
        idd = _ids_desc(ids)
        if need_bwd and 0 < B <= _mrec.BWD_HASH_MAX_BATCH:
            # the backward's hash plan runs in leading workgroups of this launch
            wsb = _mrec.lib().mrec_emb_bwd_workspace_size(bank.n_tables, B)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            desc = bank.desc()
            desc.ref()
            job = _mrec.PlanJob(ctypes.pointer(desc.struct), ctypes.pointer(idd.struct), B,
                                ws.data_ptr(), wsb, None, bank.step_counter().data_ptr())
            plan_ws = (ws, wsb)
        if B:
            _mrec.call("mrec_interact_fwd_ex", bank.desc().ref(), idd.ref(), B,
                       _mrec.ptr(dense), n_dense, dense.stride(0) if dense is not None else 0,
                       _mrec.ptr(dense_w), _mrec.ptr(bias), flags, _mrec.ptr(x0),
                       _mrec.dtype_code(x0_dtype), x0.stride(0) if x0 is not None else 0,
                       int(x0_cols), logit.data_ptr(), _mrec.ptr(fm_sum), _mrec.ptr(flag),
                       ctypes.byref(job) if job is not None else None, _mrec.stream_handle())
        if need_bwd and plan_ws is None and 0 < B <= _mrec.BWD_MAX_BATCH:
            plan_ws = _make_plan(bank, ids, B)
        _raise_if_oob(flag)
        ctx.bank, ctx.ids, ctx.B, ctx.plan_ws = bank, ids, B, plan_ws
        ctx.fm2, ctx.first_order = fm2, first_order
        # an output the model does not use (DCN-v2's logit) gets None, not a zero
        # tensor autograd would fill with a kernel of its own every step
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x0, fm_sum, dense)
        ctx.has_dense_w = dense_w is not None
        ctx.has_bias = bias is not None
        ctx.dense_w, ctx.bias = dense_w, bias
        ctx.ret_x0 = ret_x0
        if not ret_x0:
            return logit
        return x0, logit

    @staticmethod
    def backward(ctx, *grads):
        if ctx.ret_x0:
            dx0, dlogit = grads
        else:
            dx0, dlogit = None, grads[0]
        x0, fm_sum, dense = ctx.saved_tensors
        bank = ctx.bank
        if dlogit is not None:
            dlogit = dlogit.contiguous().float()
        dfm = dlogit if (ctx.fm2 and dlogit is not None) else None
        dw = dlogit if (ctx.first_order and dlogit is not None) else None
        if dx0 is not None:
            dx0 = dx0.contiguous()
        grad = None
        if bank.fused or bank.weight.requires_grad:
            grad = _backward_into_bank(bank, ctx.ids, ctx.B, ctx.plan_ws, dx=dx0, dfm=dfm,
                                       fm_sum=fm_sum, x0=x0 if dfm is not None else None, dw=dw)
        g_dense_w, g_bias = _dense_first_order_grads(ctx, dlogit, dense)
        return grad, g_dense_w, g_bias, None, None, None, None, None, None, None, None, None


def _dense_first_order_grads(ctx, dlogit, dense):
    """Gradients of the dense first-order weight and the global bias (column sums of
    dlogit), or — when both train by fused SGD — their in-place update."""
    if dlogit is None or not (ctx.has_dense_w or ctx.has_bias):
        return None, None
    from pytorchrec_amd.dense import colsum, sgd_lr
    X = dense if (ctx.has_dense_w and dense is not None) else None
    lr = sgd_lr(ctx.dense_w if X is not None else None, ctx.bias)
    if lr is not None:
        colsum(dlogit, X, want_total=ctx.has_bias,
               out=ctx.dense_w.detach() if X is not None else None,
               total=ctx.bias.detach() if ctx.has_bias else None, sgd_lr=lr)
        return None, None
    gw, gb = colsum(dlogit, X, want_total=ctx.has_bias)
    return (gw if X is not None else None), gb


def interact(bank: EmbeddingBank, ids: Sequence[torch.Tensor], dense: Optional[torch.Tensor] = None,
             dense_w: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
             fm2: bool = True, first_order: bool = True, x0_cols: int = 0,
             x0_dtype: torch.dtype = torch.bfloat16):
    """Fused DeepFM/FM/DCN input stage (see include/mrec.h ``mrec_interact_fwd``).

    Returns ``logit`` [B] (bias + dense.dense_w + FM2 + sum_f w) when ``x0_cols`` is 0,
    else ``(x0 [B, x0_cols], logit)`` with x0 = [v_0..v_{F-1} | dense | 0-pad].
    """
    ids = list(ids)
    if len(ids) != bank.n_tables:
        raise ValueError(f"expected {bank.n_tables} id tensors, got {len(ids)}")
    if first_order and not bank.has_w:
        raise ValueError("first_order needs a bank built with_first_order=True")
    if dense is not None:
        dense = dense.contiguous().float()
    from pytorchrec_amd.sharding import ShardedEmbeddingBank, sharded_interact
    if isinstance(bank, ShardedEmbeddingBank):
        return sharded_interact(bank, ids, dense, dense_w, bias, fm2, first_order, int(x0_cols),
                                x0_dtype)
    if not bank.weight.is_cuda:
        return cpu_path.interact(bank, ids, dense, dense_w, bias, fm2, first_order, x0_cols,
                                 x0_dtype)
    trigger = _trigger(bank)
    return _InteractFn.apply(bank.weight, dense_w, bias, trigger, bank, ids, dense, fm2,
                             first_order, int(x0_cols), x0_dtype, _needs_backward(bank))


def fm2_dense(v: torch.Tensor) -> torch.Tensor:
    """FM second order of a dense [B, F, D] fp32 tensor (HIP on GPU)."""
    return _Fm2Fn.apply(v) if v.is_cuda else cpu_path.fm2(v)


class _Fm2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v):
        v = v.contiguous().float()
        B, F, D = v.shape
        y = torch.empty(B, dtype=torch.float32, device=v.device)
        _mrec.call("mrec_fm2_fwd", v.data_ptr(), B, F, D, y.data_ptr(), _mrec.stream_handle())
        ctx.save_for_backward(v)
        return y

    @staticmethod
    def backward(ctx, dy):
        (v,) = ctx.saved_tensors
        B, F, D = v.shape
        dv = torch.empty_like(v)
        dy = dy.contiguous().float()
        _mrec.call("mrec_fm2_bwd", v.data_ptr(), dy.data_ptr(), B, F, D, dv.data_ptr(),
                   _mrec.stream_handle())
        return dv


def init_bank_(bank: EmbeddingBank, std: float = 0.01, generator=None, chunk_rows: int = 1 << 24):
    """normal(0, std) init in row chunks (IModel._reset_weights_fn, IModel.py:67-68);
    chunked so multi-GB banks never need a second full-size temporary."""
    with torch.no_grad():
        w = bank.weight
        for s in range(0, w.shape[0], chunk_rows):
            w[s:s + chunk_rows].normal_(0.0, std, generator=generator)
    return bank.zero_pad_()


def rows_to_bytes(bank: EmbeddingBank) -> int:
    return bank.weight.numel() * bank.weight.element_size()


__all__ = ["EmbeddingBank", "gather", "interact", "fm2_dense", "init_bank_", "rows_to_bytes"]

