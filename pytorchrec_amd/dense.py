"""Dense-tower ops: Linear(+bias)(+ReLU), DCN-v2 cross, DIN attention pooling.

One seam for the model code.  On a GPU they run on libmrec's MFMA bf16 GEMM
(``mrec_gemm``: fp32 accumulation, bias / ReLU / DCN epilogues fused, the fp32
master weights converted to bf16 by one small prep kernel, the bias gradient
carried as an extra ones column of the weight-gradient GEMM).

ReLU' is applied by the *consumer* of a ReLU output: the backward GEMM (or head
kernel) that produces d(relu output) masks it in its epilogue and stamps the
gradient tensor (``_MASK_TAG`` = (mask data_ptr, version)); the producing layer
skips its own masking only when the stamp on the incoming gradient is intact.
Autograd accumulation of several consumers' gradients bumps the version, so the
producer then masks itself (masking is idempotent) — correct in every graph,
free in the MLP chain.  On a CPU device (config C1) they are the
reference's fp32 torch ops.

Activation tensors are [M, N] views of [M, round8(N)] bf16 buffers so every
row starts 16-byte aligned.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from pytorchrec_amd import _mrec

_BF16 = torch.bfloat16


def _r8(n: int) -> int:
    return (n + 7) // 8 * 8


def _alloc(M: int, N: int, dtype, device) -> torch.Tensor:
    return torch.empty(M, _r8(N), dtype=dtype, device=device)[:, :N]


def _op(t: torch.Tensor, layout: int) -> _mrec.Operand:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("GEMM operands must be 2-D with unit inner stride")
    return _mrec.Operand(t.data_ptr(), _mrec.dtype_code(t.dtype), layout, t.stride(0))


def _split_for(M: int, N: int, K: int) -> int:
    """K slices per output tile: more while a small-output long-K GEMM (weight
    gradients) would leave most of the 256 CUs (3 workgroups each) idle."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    s = 1
    while tiles * s < 384 and K // (s + 1) >= 256 and s < 64:
        s += 1
    return s


def _split_beside(M: int, N: int, K: int, budget: int = 256) -> int:
    """K slices of a weight-gradient GEMM that shares its launch with a dx GEMM
    (448 workgroups at C2): at most ``budget`` workgroups, so the launch fits one
    residency wave (768 slots).  C2 (49 tiles, K 4096): 5 slices 138.3 us/step,
    7 slices 143.4, 4 slices +1.3 %."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    s = 1
    while tiles * (s + 1) <= budget and K // (s + 1) >= 256 and s < 64:
        s += 1
    return s


# K slices of a fused-SGD weight-gradient GEMM (0: _split_for's choice)
_DW_SPLIT = int(os.environ.get("MREC_DW_SPLIT", "0"))

_MASK_TAG = "_mrec_relu_masked"
_RELU_OUT = "_mrec_relu_out"


def _stamp(grad: torch.Tensor, mask_src: torch.Tensor) -> torch.Tensor:
    setattr(grad, _MASK_TAG, (mask_src.data_ptr(), grad._version))
    return grad


def _premasked(grad: torch.Tensor, y_ptr: int) -> bool:
    t = getattr(grad, _MASK_TAG, None)
    return t is not None and t[0] == y_ptr and t[1] == grad._version


def _is_relu_out(x: torch.Tensor) -> bool:
    return getattr(x, _RELU_OUT, False) and x.is_cuda


def gemm(A, a_layout, B, b_layout, M, N, K, *, ones_out=None, b_cols=None, bias=None, act=0,
         mul=None, add=None, aux=None, mask=None, out=None, out_dtype=_BF16, split_k=None,
         sgd_lr=None, img_row=None, img_tr=None, img_kind=0):
    """C[M, N] = epi(A[M, K] @ B[K, N]) on libmrec (see include/mrec.h mrec_gemm).
    ``ones_out`` (fp32 [M]) receives sum_k A(m, k) through an appended ones column;
    ``mask`` ([M, N] bf16) zeroes outputs where mask <= 0 (ReLU')."""
    dev = A.device
    if out is None:
        out = _alloc(M, N, out_dtype, dev)
    if split_k is None:
        split_k = _split_for(M, N + (ones_out is not None), K)
    ws_bytes = _mrec.lib().mrec_gemm_workspace_size(M, N, K, split_k)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
    epi = _mrec.Epilogue(_mrec.ptr(bias), act, _mrec.ptr(mul), mul.stride(0) if mul is not None else 0,
                         _mrec.ptr(add), add.stride(0) if add is not None else 0,
                         _mrec.ptr(aux), aux.stride(0) if aux is not None else 0,
                         _mrec.ptr(mask), mask.stride(0) if mask is not None else 0,
                         _mrec.ptr(ones_out), int(sgd_lr is not None),
                         float(sgd_lr) if sgd_lr is not None else 0.0,
                         _mrec.ptr(img_row), img_row.stride(0) if img_row is not None else 0,
                         _mrec.ptr(img_tr), img_tr.stride(0) if img_tr is not None else 0,
                         img_kind)
    a_op, b_op = _op(A, a_layout), _op(B, b_layout)
    _mrec.call("mrec_gemm", M, N, K, ctypes.byref(a_op), ctypes.byref(b_op),
               N if ones_out is not None else -1, N if b_cols is None else b_cols,
               ctypes.byref(epi), out.data_ptr(), _mrec.dtype_code(out.dtype), out.stride(0),
               split_k, _mrec.ptr(ws), ws_bytes, _mrec.stream_handle())
    return out


class _Call:
    """One GEMM of an mrec_gemm_multi launch (the ctypes structs + every tensor they
    point at, kept alive until the launch that runs it)."""

    def __init__(self, A, a_layout, B, b_layout, M, N, K, phase, *, ones_out=None, b_cols=None,
                 mask=None, out=None, out_dtype=_BF16, split_k=1, sgd_lr=None, img_row=None,
                 img_tr=None, ws=None, add=None, img_kind=0):
        dev = A.device
        if out is None:
            out = _alloc(M, N, out_dtype, dev)
        ws_bytes = _mrec.lib().mrec_gemm_workspace_size(M, N, K, split_k)
        if ws_bytes and ws is None:
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        self.out, self.ws = out, ws
        self.keep = [A, B, ones_out, mask, img_row, img_tr, out, ws, add]
        self.epi = _mrec.Epilogue(None, 0, None, 0,
                                  _mrec.ptr(add), add.stride(0) if add is not None else 0, None, 0,
                                  _mrec.ptr(mask), mask.stride(0) if mask is not None else 0,
                                  _mrec.ptr(ones_out), int(sgd_lr is not None),
                                  float(sgd_lr) if sgd_lr is not None else 0.0,
                                  _mrec.ptr(img_row), img_row.stride(0) if img_row is not None else 0,
                                  _mrec.ptr(img_tr), img_tr.stride(0) if img_tr is not None else 0,
                                  img_kind)
        self.a, self.b = _op(A, a_layout), _op(B, b_layout)
        self.args = (M, N, K, N if ones_out is not None else -1, N if b_cols is None else b_cols,
                     out.data_ptr(), _mrec.dtype_code(out.dtype), out.stride(0), split_k,
                     _mrec.ptr(ws), ws_bytes)
        self.phase = phase
        self.writes = {p for p in (out.data_ptr(), _mrec.ptr(ones_out), _mrec.ptr(img_row),
                                   _mrec.ptr(img_tr)) if p}
        self.reads = {A.data_ptr(), B.data_ptr()} | ({add.data_ptr()} if add is not None else set())

    def with_phase(self, phase):
        c = object.__new__(_Call)
        c.__dict__.update(self.__dict__)
        c.phase = phase
        return c

    def struct(self) -> _mrec.GemmCall:
        M, N, K, ones, bcols, C, cdt, ldc, sk, ws, wsb = self.args
        return _mrec.GemmCall(M, N, K, ctypes.pointer(self.a), ctypes.pointer(self.b), ones, bcols,
                              ctypes.pointer(self.epi), C, cdt, ldc, sk, ws, wsb, self.phase)


_PENDING = []  # deferred split-K reductions (fused SGD of a layer's W, b and images)
CO_REDUCE_MAX = 6  # reductions one embedding-update launch takes along (gemm_common.h kMaxCoReduce)

# measurement hook (bench.py): when a dict, the tower launches of eager steps are
# bracketed by HIP events on their stream: {name: [(start, end), ...]}
KERNEL_EVENTS = None


class _timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if KERNEL_EVENTS is not None:
            # keep the queue busy (~80 us spin) so the start event and the launch are
            # both queued when the GPU reaches them: the host's launch latency of an
            # eager step is then outside the bracket
            torch.cuda._sleep(200000)
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if KERNEL_EVENTS is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            KERNEL_EVENTS.setdefault(self.name, []).append((self.e0, e1))
        return False


# the batch feed's copy of a later batch (an mrec_feed_job, loader.capture_steps),
# taken by the next mrec_tower_dw launch: its PCIe reads then run in extra workgroups
# beside the L2-bound weight-gradient tiles instead of on the step's critical path
_FEED_JOB = []


def set_feed_job(job):
    _FEED_JOB[:] = [job]


def take_feed_job():
    job = _FEED_JOB[0] if _FEED_JOB else None
    _FEED_JOB.clear()
    return job


def launch_multi(calls):
    """Run ``calls`` plus the pending deferred reductions in as few launches as
    possible (<= 4 problems each; a pending job that writes what a call reads is
    flushed first)."""
    global _PENDING
    pend = _PENDING
    reads = set().union(*[c.reads for c in calls]) if calls else set()
    if any(p.writes & reads for p in pend):
        _run(pend)
        pend = []
    jobs = list(calls) + pend
    _PENDING = []
    for i in range(0, len(jobs), 4):
        _run(jobs[i:i + 4])


class _HeadFinish:
    """A deferred mrec_ctr_head_finish in SGD-update mode (the head's W, b and side
    linear ws, b2): run by spare workgroups of the next GEMM launch, or on its own
    at the end of the backward."""

    def __init__(self, part, B, H, ns, g, lr, w, bias, ws, b2, grads=None):
        self.keep = [part, g, w, bias, ws, b2, grads]
        if grads is None:  # SGD update in place
            self.struct = _mrec.HeadFinishJob(part.data_ptr(), part.stride(0), B, H, ns,
                                              _mrec.ptr(g), 1, float(lr), w.data_ptr(),
                                              _mrec.ptr(bias), _mrec.ptr(ws), _mrec.ptr(b2),
                                              None, None, None, None)
        else:  # gradients into the data-parallel flat buffer views
            self.struct = _mrec.HeadFinishJob(part.data_ptr(), part.stride(0), B, H, ns,
                                              _mrec.ptr(g), 0, 0.0, None, None, None, None,
                                              *[_mrec.ptr(t) for t in grads])

    def run(self):
        j = self.struct
        _mrec.call("mrec_ctr_head_finish", j.part, j.ldp, j.batch, j.H, j.ns, j.g, j.update, j.lr,
                   j.w, j.bias, j.ws, j.b2, j.dw_out, j.db_out, j.dws_out, j.db2_out,
                   _mrec.stream_handle())


_FINISH = []


def defer_head_finish(fin: _HeadFinish):
    _flush_finish()
    _FINISH.append(fin)
    torch.autograd.Variable._execution_engine.queue_callback(flush_pending)


def _flush_finish():
    while _FINISH:
        _FINISH.pop(0).run()


def _run(jobs):
    if not jobs:
        return
    arr = (_mrec.GemmCall * len(jobs))(*[j.struct() for j in jobs])
    fin = _FINISH.pop(0) if _FINISH else None
    if fin is None:
        _mrec.call("mrec_gemm_multi", len(jobs), arr, _mrec.stream_handle())
        return
    _mrec.call("mrec_gemm_multi_ex", len(jobs), arr, None, ctypes.byref(fin.struct),
               _mrec.stream_handle())


def flush_pending():
    """Apply every deferred reduction now (queued as an autograd end-of-backward
    callback whenever one is deferred, so a backward pass never ends with work
    pending)."""
    global _PENDING
    pend, _PENDING = _PENDING, []
    for i in range(0, len(pend), 4):
        _run(pend[i:i + 4])
    _flush_finish()


def take_pending(n: int):
    """Remove and return up to ``n`` deferred reductions, for a launch that runs
    them beside its own work (``mrec_emb_bwd_apply_ex``)."""
    global _PENDING
    jobs, _PENDING = _PENDING[:n], _PENDING[n:]
    return jobs


def _defer(call: "_Call"):
    _PENDING.append(call.with_phase(_mrec.GEMM_REDUCE))
    torch.autograd.Variable._execution_engine.queue_callback(flush_pending)


def weight_prep(W: torch.Tensor, row: bool = True, tr: bool = True):
    """bf16 images of an fp32 [N, K] weight: row [N, r8(K)] and W^T [K, r8(N)]."""
    W = _weight_f32(W)
    N, K = W.shape
    wr = torch.empty(N, _r8(K), dtype=_BF16, device=W.device) if row else None
    wt = torch.empty(K, _r8(N), dtype=_BF16, device=W.device) if tr else None
    _mrec.call("mrec_weight_prep", W.data_ptr(), N, K, W.stride(0), _mrec.ptr(wr),
               wr.stride(0) if wr is not None else 0, _mrec.ptr(wt),
               wt.stride(0) if wt is not None else 0, _mrec.stream_handle())
    return wr, wt


# bf16 images of an fp32 master weight, cached on the Parameter per kind:
#   "rowtr": row-major W and W^T (operands of mrec_gemm);
#   "tower": the MFMA-fragment images of the fused tower (mrec_tower_fwd_bwd).
# An entry is valid while (weight._version, weight._mrec_gen) is unchanged: torch
# modifying the weight bumps the version; a kernel updating it in place (fused
# SGD) re-emits the images it was handed and ``images_updated`` bumps the
# generation and re-stamps that kind, so only the other kind goes stale.
_IMG_ATTR = {"rowtr": "_mrec_img", "tower": "_mrec_timg"}


def _img_state(weight):
    return weight._version, getattr(weight, "_mrec_gen", 0)


def cached_images(weight: torch.Tensor, kind: str):
    """The valid cached ``kind`` images of ``weight`` (a pair) or None."""
    c = getattr(weight, _IMG_ATTR[kind], None)
    if (c is not None and (c[0], c[1]) == _img_state(weight) and c[2].device == weight.device):
        return c[2], c[3]
    return None


def images_updated(weight: torch.Tensor, kind: str):
    """An in-place update of ``weight`` (fused SGD) has been enqueued that also
    rewrites its ``kind`` images: they stay valid, every other kind is stale."""
    gen = getattr(weight, "_mrec_gen", 0) + 1
    weight._mrec_gen = gen
    attr = _IMG_ATTR[kind]
    c = getattr(weight, attr, None)
    if c is not None:
        setattr(weight, attr, (weight._version, gen) + tuple(c[2:]))


def weight_images(weight: torch.Tensor):
    """(row, transposed) bf16 images of a Parameter, cached on it and rebuilt only
    when the weight changed since (see ``_IMG_ATTR``)."""
    c = cached_images(weight, "rowtr")
    if c is not None and c[0].shape[0] == weight.shape[0]:
        return c
    wr, wt = weight_prep(weight)
    weight._mrec_img = _img_state(weight) + (wr, wt)
    return wr, wt


def tower_images(weight: torch.Tensor):
    """(fwd, bwd) MFMA-fragment images of a Linear weight [N, K] for the fused
    tower (csrc/tower_common.h), cached like ``weight_images``.  Zero-initialised:
    the prep writes only real elements, the pad entries stay zero."""
    c = cached_images(weight, "tower")
    if c is not None:
        return c
    W = _weight_f32(weight)
    N, K = W.shape
    lib = _mrec.lib()
    pf = torch.zeros(int(lib.mrec_tower_image_elems(N, K, 0)), dtype=_BF16, device=W.device)
    pb = torch.zeros(int(lib.mrec_tower_image_elems(N, K, 1)), dtype=_BF16, device=W.device)
    _mrec.call("mrec_tower_weight_prep", W.data_ptr(), N, K, W.stride(0), pf.data_ptr(),
               pb.data_ptr(), _mrec.stream_handle())
    weight._mrec_timg = _img_state(weight) + (pf, pb)
    return pf, pb


def sgd_lr(*params) -> Optional[float]:
    """The learning rate when every given parameter (None entries ignored) is
    trained by plain SGD fused into its backward (IModel.compile marks them), with
    one common lr; else None (the gradient is returned to the optimizer)."""
    lr = None
    for p in params:
        if p is None:
            continue
        g = getattr(p, "_mrec_sgd_group", None)
        if g is None:
            return None
        if lr is None:
            lr = float(g["lr"])
        elif float(g["lr"]) != lr:
            return None
    return lr


def dp_grads(*params):
    """Data-parallel flat-gradient views of ``params`` (None entries ignored), or
    None unless every given parameter has one (``IModel.distribute`` assigns them:
    the backward kernels write the gradients there, IModel all-reduces the flat
    buffer once and applies SGD with one mrec_sgd_multi launch)."""
    out = []
    for p in params:
        if p is None:
            out.append(None)
            continue
        g = getattr(p, "_mrec_dp_grad", None)
        if g is None:
            return None
        out.append(g)
    return out


def _bf16_rows(t: torch.Tensor) -> torch.Tensor:
    """bf16 [M, N] with 16-byte aligned rows (what mrec_gemm requires); copies into
    an r8-padded buffer only when the input is not already laid out that way."""
    if (t.dtype == _BF16 and t.stride(-1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0):
        return t
    M, N = t.shape
    if N % 8:  # the pad columns are read by 16-B staging: they must be zero
        out = torch.zeros(M, _r8(N), dtype=_BF16, device=t.device)[:, :N]
    else:
        out = _alloc(M, N, _BF16, t.device)
    out.copy_(t)
    return out


def _weight_f32(w: torch.Tensor) -> torch.Tensor:
    w = w.detach()
    if w.dtype != torch.float32:
        w = w.float()
    return w if w.stride(1) == 1 else w.contiguous()


class _LinearFn(torch.autograd.Function):
    """y = act(x[:, :K] W^T + b) with W [N, K] fp32 (nn.Linear layout).
    x_relu: x is a ReLU output, so dx is masked by x in the dx GEMM's epilogue.
    With fused SGD (sgd_lr) the weight-gradient GEMM applies W -= lr dW, b -= lr db
    and rewrites the bf16 images; no gradient is returned."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, out_dtype, x_relu: bool):
        x = _bf16_rows(x)
        M, K_x = x.shape
        N, K = weight.shape
        flush_pending()
        wr, wt = weight_images(weight)
        b = bias.detach().float().contiguous() if bias is not None else None
        y = gemm(x, _mrec.LAYOUT_ROW, wr[:, :K], _mrec.LAYOUT_ROW, M, N, K, bias=b,
                 act=_mrec.ACT_RELU if relu else _mrec.ACT_NONE, out_dtype=out_dtype)
        ctx.save_for_backward(x, y if relu else None)
        ctx.relu, ctx.has_bias, ctx.NK, ctx.x_relu = relu, bias is not None, (N, K), x_relu
        ctx.y_ptr = y.data_ptr()
        ctx.weight, ctx.bias, ctx.wr, ctx.wt = weight, bias, wr, wt
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        M, K_x = x.shape
        N, K = ctx.NK
        if ctx.relu and not _premasked(dy, ctx.y_ptr):
            dy = torch.where(y > 0, dy.to(y.dtype), torch.zeros((), dtype=y.dtype, device=y.device))
        dy = _bf16_rows(dy)
        dx = dW = db = None
        need_w = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        lr = sgd_lr(ctx.weight, ctx.bias) if need_w else None
        dpg = dp_grads(ctx.weight, ctx.bias) if need_w and lr is None else None
        if lr is not None or dpg is not None:
            # one launch: dx GEMM + dW partial slabs (+ earlier layers' deferred dW
            # reductions); this layer's reduction + SGD runs in the next launch.
            # Data-parallel: the reduction writes dW / db into the flat gradient
            # buffer that IModel all-reduces (then one mrec_sgd_multi updates)
            calls = []
            if ctx.needs_input_grad[0]:
                cdx = _Call(dy, _mrec.LAYOUT_ROW, ctx.wt, _mrec.LAYOUT_ROW, M, K_x, N,
                            _mrec.GEMM_FULL, b_cols=K, mask=x if ctx.x_relu else None)
                calls.append(cdx)
                dx = cdx.out
            sk = _DW_SPLIT or _split_beside(N, K + 1, M)
            if dpg is not None:
                cdw = _Call(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M,
                            _mrec.GEMM_PARTIAL if sk > 1 else _mrec.GEMM_FULL,
                            ones_out=dpg[1], out=dpg[0], out_dtype=torch.float32, split_k=sk)
            else:
                cdw = _Call(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M,
                            _mrec.GEMM_PARTIAL if sk > 1 else _mrec.GEMM_FULL,
                            ones_out=ctx.bias.detach() if ctx.has_bias else None,
                            out=ctx.weight.detach(), out_dtype=torch.float32, split_k=sk,
                            sgd_lr=lr, img_row=ctx.wr, img_tr=ctx.wt)
                images_updated(ctx.weight, "rowtr")
            if sk > 1:
                launch_multi(calls + [cdw])
                _defer(cdw)
            elif dpg is not None:  # plain dW output: independent of the dx GEMM
                launch_multi(calls + [cdw])
            else:  # the dW epilogue rewrites wt, which the dx GEMM reads: two launches
                launch_multi(calls)
                launch_multi([cdw])
            if ctx.x_relu and dx is not None:
                _stamp(dx, x)
            return dx, None, None, None, None, None
        if ctx.needs_input_grad[0]:
            # dx[m, k] = sum_n dZ[m, n] W[n, k]; B(k'=n, col=k) = W^T[k*ld + n] -> ROW
            flush_pending()
            dx = gemm(dy, _mrec.LAYOUT_ROW, ctx.wt, _mrec.LAYOUT_ROW, M, K_x, N, b_cols=K,
                      mask=x if ctx.x_relu else None, out_dtype=_BF16)
            if ctx.x_relu:
                _stamp(dx, x)
        if need_w:
            # dW[n, k] = sum_m dZ[m, n] x[m, k]: A(i=n, red=m) = dy[m*ld + n] -> COL,
            # B(red=m, col=k) = x[m*ld + k] -> COL; ones column -> db
            dW = torch.empty(N, K, dtype=torch.float32, device=dy.device)
            db = torch.empty(N, dtype=torch.float32, device=dy.device) if ctx.has_bias else None
            gemm(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M, ones_out=db, out=dW)
        return dx, dW, db, None, None, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
           act: Optional[str] = None, out_dtype=_BF16) -> torch.Tensor:
    """y = act(x W^T + b), W stored [out, in] like nn.Linear (Dense.py:12).  x may
    carry zero pad columns beyond in_features; they are ignored (and get a zero
    gradient)."""
    if not x.is_cuda:
        k = weight.shape[1]
        xx = x[:, :k] if x.shape[1] > k else x
        y = F.linear(xx.float(), weight.float(), None if bias is None else bias.float())
        return torch.relu(y) if act == "relu" else y
    y = _LinearFn.apply(x, weight, bias, act == "relu", out_dtype, _is_relu_out(x))
    if act == "relu":
        setattr(y, _RELU_OUT, True)
    return y


class _CrossFn(torch.autograd.Function):
    """DCN-v2 layer x_{l+1} = x0 * (x_l W^T + b) + x_l (one GEMM, epilogue fused;
    z = x_l W^T + b kept for the backward)."""

    @staticmethod
    def forward(ctx, x0, xl, weight, bias):
        x0, xl = _bf16_rows(x0), _bf16_rows(xl)
        M = xl.shape[0]
        d = weight.shape[0]
        wr, wt = weight_images(weight)
        b = bias.detach().float().contiguous() if bias is not None else None
        z = _alloc(M, d, _BF16, xl.device)
        out = gemm(xl, _mrec.LAYOUT_ROW, wr[:, :d], _mrec.LAYOUT_ROW, M, d, d, bias=b, mul=x0,
                   add=xl, aux=z)
        ctx.save_for_backward(x0, xl, z)
        ctx.has_bias = bias is not None
        ctx.weight, ctx.bias, ctx.wr, ctx.wt = weight, bias, wr, wt
        return out

    @staticmethod
    def backward(ctx, g):
        x0, xl, z = ctx.saved_tensors
        wt = ctx.wt
        g = _bf16_rows(g)
        M = g.shape[0]
        d = z.shape[1]
        # dz = g * x0; dx_l = dz W + g; dW = dz^T x_l; db = sum dz
        dz = _alloc(M, d, _BF16, g.device)
        torch.mul(g[:, :d], x0[:, :d], out=dz)
        if dz.stride(0) > d:
            dz.as_strided((M, dz.stride(0) - d), (dz.stride(0), 1), d).zero_()
        dxl = gemm(dz, _mrec.LAYOUT_ROW, wt, _mrec.LAYOUT_ROW, M, xl.shape[1], d, b_cols=d,
                   add=_pad_cols(g, xl.shape[1]))
        dW = db = None
        lr = sgd_lr(ctx.weight, ctx.bias)
        if lr is not None:
            gemm(dz, _mrec.LAYOUT_COL, xl, _mrec.LAYOUT_COL, d, d, M,
                 ones_out=ctx.bias.detach() if ctx.has_bias else None, out=ctx.weight.detach(),
                 out_dtype=torch.float32, sgd_lr=lr, img_row=ctx.wr, img_tr=ctx.wt)
            images_updated(ctx.weight, "rowtr")
        else:
            dW = torch.empty(d, d, dtype=torch.float32, device=g.device)
            db = torch.empty(d, dtype=torch.float32, device=g.device) if ctx.has_bias else None
            gemm(dz, _mrec.LAYOUT_COL, xl, _mrec.LAYOUT_COL, d, d, M, ones_out=db, out=dW)
        dx0 = (g.float() * z.float()).to(_BF16)
        if x0.shape[1] > d:
            dx0 = F.pad(dx0, (0, x0.shape[1] - d))
        return dx0, dxl, dW, db


class _CrossNetFn(torch.autograd.Function):
    """The whole DCN-v2 cross network x_{l+1} = x0 * (x_l W_l^T + b_l) + x_l,
    l = 0..L-1, as one autograd node: forward = one fused GEMM per layer; backward
    per layer = ONE elementwise kernel (mrec_dcn_cross_bwd_prep: dz = g*x0 and the
    fp32 sum over layers of g*z, i.e. x0's multiplier gradient) + the dx_l GEMM
    (layer 0 adds that sum, so its output is dx0) + the dW GEMM (fused SGD when
    compiled with plain SGD, data-parallel gradient views, else returned)."""

    @staticmethod
    def forward(ctx, x0, n, *params):
        weights, biases = params[:n], params[n:]
        x0 = _bf16_rows(x0)
        xl = x0
        saved = []
        for W, b in zip(weights, biases):
            M = xl.shape[0]
            d = W.shape[0]
            wr, wt = weight_images(W)
            bb = b.detach().float().contiguous() if b is not None else None
            z = _alloc(M, d, _BF16, xl.device)
            out = gemm(xl, _mrec.LAYOUT_ROW, wr[:, :d], _mrec.LAYOUT_ROW, M, d, d, bias=bb,
                       mul=x0, add=xl, aux=z)
            saved.append((xl, z, wr, wt))
            xl = out
        ctx.x0, ctx.saved, ctx.weights, ctx.biases = x0, saved, weights, biases
        return xl

    @staticmethod
    def backward(ctx, g):
        x0, saved = ctx.x0, ctx.saved
        L = len(saved)
        g = _bf16_rows(g)
        M = g.shape[0]
        d = saved[0][1].shape[1]
        acc = torch.empty(M, _r8(d), dtype=torch.float32, device=g.device)
        dWs, dbs = [None] * L, [None] * L
        for l in reversed(range(L)):
            xl, z, wr, wt = saved[l]
            W, b = ctx.weights[l], ctx.biases[l]
            dz = _alloc(M, d, _BF16, g.device)
            addend = _alloc(M, xl.shape[1], _BF16, g.device) if l == 0 else None
            _mrec.call("mrec_dcn_cross_bwd_prep", M, d, g.data_ptr(), g.stride(0),
                       x0.data_ptr(), x0.stride(0), z.data_ptr(), z.stride(0), dz.data_ptr(),
                       dz.stride(0), acc.data_ptr(), acc.stride(0), int(l == L - 1),
                       _mrec.ptr(addend), addend.stride(0) if addend is not None else 0,
                       _mrec.stream_handle())
            # dx_l = dz W (+ g: x_l feeds the residual; layer 0: + sum_l g_l*z_l too)
            add = addend if l == 0 else _pad_cols(g, xl.shape[1])
            lr = sgd_lr(W, b)
            dpg = dp_grads(W, b) if lr is None else None
            if lr is not None or dpg is not None:
                # one launch: dx GEMM + dW split-K slabs (+ the previous layer's deferred
                # dW reduction); this layer's reduction rides in the next launch
                cdx = _Call(dz, _mrec.LAYOUT_ROW, wt, _mrec.LAYOUT_ROW, M, xl.shape[1], d,
                            _mrec.GEMM_FULL, b_cols=d, add=add)
                sk = _DW_SPLIT or _split_beside(d, d + 1, M)
                ph = _mrec.GEMM_PARTIAL if sk > 1 else _mrec.GEMM_FULL
                if dpg is not None:
                    cdw = _Call(dz, _mrec.LAYOUT_COL, xl, _mrec.LAYOUT_COL, d, d, M, ph,
                                ones_out=dpg[1], out=dpg[0], out_dtype=torch.float32, split_k=sk)
                else:
                    cdw = _Call(dz, _mrec.LAYOUT_COL, xl, _mrec.LAYOUT_COL, d, d, M, ph,
                                ones_out=b.detach() if b is not None else None, out=W.detach(),
                                out_dtype=torch.float32, split_k=sk, sgd_lr=lr, img_row=wr,
                                img_tr=wt)
                    images_updated(W, "rowtr")
                if sk > 1:
                    launch_multi([cdx, cdw])
                    _defer(cdw)
                elif dpg is not None:
                    launch_multi([cdx, cdw])
                else:  # the dW epilogue rewrites wt, which the dx GEMM reads
                    launch_multi([cdx])
                    launch_multi([cdw])
                g = cdx.out
                continue
            flush_pending()
            gx = gemm(dz, _mrec.LAYOUT_ROW, wt, _mrec.LAYOUT_ROW, M, xl.shape[1], d, b_cols=d,
                      add=add)
            dWs[l] = torch.empty(d, d, dtype=torch.float32, device=g.device)
            dbs[l] = torch.empty(d, dtype=torch.float32, device=g.device) if b is not None else None
            gemm(dz, _mrec.LAYOUT_COL, xl, _mrec.LAYOUT_COL, d, d, M, ones_out=dbs[l], out=dWs[l])
            g = gx
        ctx.saved = None
        return (g, None, *dWs, *dbs)


def cross_net(x0: torch.Tensor, weights: Sequence[torch.Tensor],
              biases: Sequence[Optional[torch.Tensor]]) -> torch.Tensor:
    """A stack of DCN-v2 cross layers over x0 (one autograd node on the GPU)."""
    if not x0.is_cuda or any(b is None for b in biases):
        x = x0
        for W, b in zip(weights, biases):
            x = cross(x0, x, W, b)
        return x
    return _CrossNetFn.apply(x0, len(weights), *weights, *biases)


def _pad_cols(t: torch.Tensor, n: int) -> torch.Tensor:
    if t.shape[1] == n:
        return t
    out = torch.zeros(t.shape[0], _r8(n), dtype=t.dtype, device=t.device)[:, :n]
    out[:, :t.shape[1]] = t
    return out


def cross(x0: torch.Tensor, xl: torch.Tensor, weight: torch.Tensor,
          bias: Optional[torch.Tensor]) -> torch.Tensor:
    """DCN-v2 cross layer x_{l+1} = x0 * (W x_l + b) + x_l."""
    d = weight.shape[1]
    if not xl.is_cuda:
        x0c = x0[:, :d].float()
        xlc = xl[:, :d].float()
        return x0c * F.linear(xlc, weight.float(), None if bias is None else bias.float()) + xlc
    return _CrossFn.apply(x0, xl, weight, bias)


def din_attention(q: torch.Tensor, k: torch.Tensor, valid: torch.Tensor, att_mlp,
                  att_out: torch.nn.Linear):
    """DIN target attention (torch ops; the CPU path and the reference restatement):
    s_j = att_out(att_mlp([q, k_j, q-k_j, q*k_j])); a = softmax over valid j
    (invalid -> -inf, SASRec.py:26-29); u = sum_j a_j k_j.
    q [B, E], k [B, L, E], valid [B, L] bool -> u [B, E] (fp32)."""
    B, L, E = k.shape
    qb = q.unsqueeze(1).expand(B, L, E).to(k.dtype)
    feat = torch.cat([qb, k, qb - k, qb * k], dim=-1).reshape(B * L, 4 * E)
    h = att_mlp(feat)
    s = linear(h, att_out.weight, att_out.bias, out_dtype=torch.float32).float().reshape(B, L)
    s = s.masked_fill(~valid, float("-inf"))
    a = torch.softmax(s, dim=-1)
    return (a.unsqueeze(-1) * k.float()).sum(1)


class _DinState:
    """Carries the pooling backward's dk / dq pieces to the feature backward (the
    pooling backward always runs first: its ds feeds the attention MLP backward)."""


class _DinFeatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, st: _DinState, L: int):
        B, E = q.shape
        feat = _alloc(B * L, 4 * E, _BF16, q.device)
        _mrec.call("mrec_din_feat_fwd", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), B, L,
                   E, feat.data_ptr(), feat.stride(0), _mrec.stream_handle())
        ctx.save_for_backward(q, k)
        ctx.st, ctx.L = st, L
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        q, k = ctx.saved_tensors
        st = ctx.st
        B, E = q.shape
        dfeat = _bf16_rows(dfeat)
        dq = torch.empty(B, E, dtype=torch.float32, device=q.device)
        _mrec.call("mrec_din_feat_bwd", dfeat.data_ptr(), dfeat.stride(0), st.dtop.data_ptr(),
                   st.dtop.stride(0), q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), B,
                   ctx.L, E, st.dk.data_ptr(), st.dk.stride(0), dq.data_ptr(), dq.stride(0),
                   _mrec.stream_handle())
        dk = st.dk
        del st.dk, st.dtop
        return dq, dk, None, None


class _DinPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, q, k, his, st: _DinState, L: int):
        B, E = q.shape
        a = torch.empty(B, L, dtype=torch.float32, device=q.device)
        top = _alloc(B, 2 * E, _BF16, q.device)
        his = his.to(torch.int32)
        _mrec.call("mrec_din_pool_fwd", s.data_ptr(), s.stride(0), his.data_ptr(), his.stride(0),
                   q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), B, L, E, a.data_ptr(),
                   top.data_ptr(), top.stride(0), _mrec.stream_handle())
        ctx.save_for_backward(a, k)
        ctx.st, ctx.L, ctx.E, ctx.s_shape = st, L, E, s.shape
        return top

    @staticmethod
    def backward(ctx, dtop):
        a, k = ctx.saved_tensors
        st = ctx.st
        B, L, E = a.shape[0], ctx.L, ctx.E
        dtop = _bf16_rows(dtop)
        ds = torch.empty(B * L, 1, dtype=torch.float32, device=a.device)
        dk = torch.empty(B * L, E, dtype=torch.float32, device=a.device)
        _mrec.call("mrec_din_pool_bwd", dtop.data_ptr(), dtop.stride(0), a.data_ptr(), k.data_ptr(),
                   k.stride(0), B, L, E, ds.data_ptr(), dk.data_ptr(), dk.stride(0),
                   _mrec.stream_handle())
        st.dk, st.dtop = dk, dtop
        return ds, None, None, None, None, None


class _DinRowsFeatFn(torch.autograd.Function):
    """_DinFeatFn over the gathered rows [q (B) | k (B L)] as ONE input: the backward
    returns the rows' bf16 gradient from one kernel (mrec_din_feat_bwd_rows), so
    autograd adds no slice-backward zero fills, copies or dtype casts."""

    @staticmethod
    def forward(ctx, rows, B: int, st: _DinState, L: int):
        q, k = rows[:B], rows[B:]
        E = rows.shape[1]
        feat = _alloc(B * L, 4 * E, _BF16, rows.device)
        _mrec.call("mrec_din_feat_fwd", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), B, L,
                   E, feat.data_ptr(), feat.stride(0), _mrec.stream_handle())
        ctx.save_for_backward(rows)
        ctx.st, ctx.L, ctx.B = st, L, B
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        rows, = ctx.saved_tensors
        st, B, L = ctx.st, ctx.B, ctx.L
        q, k = rows[:B], rows[B:]
        E = rows.shape[1]
        dfeat = _bf16_rows(dfeat)
        d_rows = torch.empty_like(rows)
        _mrec.call("mrec_din_feat_bwd_rows", dfeat.data_ptr(), dfeat.stride(0), st.dtop.data_ptr(),
                   st.dtop.stride(0), q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), B, L, E,
                   st.dk.data_ptr(), st.dk.stride(0), d_rows.data_ptr(), d_rows.stride(0),
                   _mrec.stream_handle())
        del st.dk, st.dtop
        return d_rows, None, None, None


# opt-in (MREC_DIN_TOWER=1): measured at C4 the score tower is slower than the
# GEMMs (fwd 279, bwd 527, weight gradients 213 us vs ~360 us for the GEMM path in
# all): 12,800 16-row workgroups at 2 per CU run 25 residency rounds of the tower's
# latency chain, and the k-fragment images of 204,800 rows go through HBM
DIN_TOWER = os.environ.get("MREC_DIN_TOWER", "0") == "1"


def _din_scores(feat: torch.Tensor, att_mlp, att_out: torch.nn.Linear) -> torch.Tensor:
    """Attention-unit scores [B L, 1] fp32: the attention MLP's GEMMs + Linear(h, 1),
    or the score tower (one launch each way) with MREC_DIN_TOWER=1."""
    if DIN_TOWER and tower_supported(feat, att_mlp, att_out):
        return score_tower(feat, att_mlp, att_out).reshape(-1, 1)
    h = att_mlp(feat)
    return linear(h, att_out.weight, att_out.bias, out_dtype=torch.float32)


# the fused attention unit (mrec_din_att_*, din_att.hip) is the default for the
# compiled shapes; MREC_DIN_FUSED=0 selects the layered kernels (A/B, parity tests)
DIN_FUSED = os.environ.get("MREC_DIN_FUSED", "1") == "1"


def _din_att_linears(att_mlp, att_out):
    lins = [m for m in att_mlp.modules() if isinstance(m, torch.nn.Linear)]
    return lins + [att_out]


def din_att_supported(E: int, att_mlp, att_out: torch.nn.Linear) -> bool:
    """True when the fused attention unit covers this block: two ReLU Dense layers
    + Linear(H2, 1), all with bias, no active dropout, a compiled (E, H1, H2)."""
    lins = _din_att_linears(att_mlp, att_out)
    if len(lins) != 3 or any(m.bias is None for m in lins) or lins[2].out_features != 1:
        return False
    if att_mlp.training and any(isinstance(m, torch.nn.Dropout) and m.p > 0
                                for m in att_mlp.modules()):
        return False
    H1, H2 = lins[0].out_features, lins[1].out_features
    if (lins[0].in_features != 4 * E or lins[1].in_features != H1
            or lins[2].in_features != H2):
        return False
    return bool(_mrec.lib().mrec_din_att_supported(E, H1, H2))


def _weights_changed(*params):
    """An in-place kernel update of these fp32 masters that re-emitted no image:
    every cached bf16 image kind goes stale."""
    for p in params:
        p._mrec_gen = getattr(p, "_mrec_gen", 0) + 1


class _DinAttFn(torch.autograd.Function):
    """The whole DIN attention unit over the gathered rows [q (B) | k (B L)]: one
    forward launch (features, MLP, scores, masked softmax, pooling -> top) and one
    backward launch (the rows' bf16 gradient + weight-gradient partials) plus the
    partials' fixed-order sum, which applies the fused SGD when the optimizer is
    plain SGD (sgd_lr) or hands the gradients to it."""

    @staticmethod
    def forward(ctx, rows, his, B: int, L: int, w1, b1, w2, b2, w3, b3):
        E = rows.shape[1]
        H1, H2 = w1.shape[0], w2.shape[0]
        ws = [_weight_f32(w1), b1.detach().float().contiguous(), _weight_f32(w2),
              b2.detach().float().contiguous(), w3.detach().float().reshape(-1).contiguous(),
              b3.detach().float().contiguous()]
        his = his.to(torch.int32)
        if his.stride(1) != 1:
            his = his.contiguous()
        a = torch.empty(B, L, dtype=torch.float32, device=rows.device)
        top = _alloc(B, 2 * E, _BF16, rows.device)
        _mrec.call("mrec_din_att_fwd", rows.data_ptr(), rows.stride(0), his.data_ptr(),
                   his.stride(0), B, L, E, ws[0].data_ptr(), ws[0].stride(0), ws[1].data_ptr(),
                   H1, ws[2].data_ptr(), ws[2].stride(0), ws[3].data_ptr(), H2, ws[4].data_ptr(),
                   ws[5].data_ptr(), a.data_ptr(), top.data_ptr(), top.stride(0),
                   _mrec.stream_handle())
        ctx.save_for_backward(rows, a)
        ctx.ws, ctx.params, ctx.B, ctx.L = ws, (w1, b1, w2, b2, w3, b3), B, L
        return top

    @staticmethod
    def backward(ctx, dtop):
        rows, a = ctx.saved_tensors
        ws, params, B, L = ctx.ws, ctx.params, ctx.B, ctx.L
        E = rows.shape[1]
        H1, H2 = params[0].shape[0], params[2].shape[0]
        dtop = _bf16_rows(dtop)
        d_rows = _alloc(rows.shape[0], E, _BF16, rows.device)
        lib = _mrec.lib()
        parts = int(lib.mrec_din_att_parts(B))
        P = int(lib.mrec_din_att_param_count(E, H1, H2))
        part = torch.empty(parts, P, dtype=torch.float32, device=rows.device)
        st = _mrec.stream_handle()
        _mrec.call("mrec_din_att_bwd", rows.data_ptr(), rows.stride(0), B, L, E,
                   ws[0].data_ptr(), ws[0].stride(0), ws[1].data_ptr(), H1, ws[2].data_ptr(),
                   ws[2].stride(0), ws[3].data_ptr(), H2, ws[4].data_ptr(), ws[5].data_ptr(),
                   a.data_ptr(), dtop.data_ptr(), dtop.stride(0), d_rows.data_ptr(),
                   d_rows.stride(0), part.data_ptr(), parts, st)
        ctx.ws = None
        w1, b1, w2, b2, w3, b3 = params
        lr = sgd_lr(*params)
        inplace = (lr is not None and all(p.dtype == torch.float32 and p.is_contiguous()
                                          for p in params))
        if inplace:
            _mrec.call("mrec_din_att_wgrad", part.data_ptr(), parts, E, H1, H2, None, lr,
                       w1.data_ptr(), w1.stride(0), b1.data_ptr(), w2.data_ptr(), w2.stride(0),
                       b2.data_ptr(), w3.data_ptr(), b3.data_ptr(), st)
            _weights_changed(*params)
            return d_rows, None, None, None, None, None, None, None, None, None
        g = torch.empty(P, dtype=torch.float32, device=rows.device)
        _mrec.call("mrec_din_att_wgrad", part.data_ptr(), parts, E, H1, H2, g.data_ptr(), 0.0,
                   None, 0, None, None, 0, None, None, None, st)
        gw1, gw2, gb1, gb2, gw3, gb3 = torch.split(g, [H1 * 4 * E, H2 * H1, H1, H2, H2, 1])
        grads = [t.view_as(p) for t, p in zip((gw1, gb1, gw2, gb2, gw3, gb3), params)]
        dpg = dp_grads(*params)
        if dpg is not None:  # data parallel: into the flat buffer IModel all-reduces
            for dst, src in zip(dpg, grads):
                dst.copy_(src.view_as(dst))
            return d_rows, None, None, None, None, None, None, None, None, None
        return (d_rows, None, None, None, *grads)


def din_attention_top_rows(rows: torch.Tensor, B: int, his: torch.Tensor, att_mlp,
                           att_out: torch.nn.Linear) -> torch.Tensor:
    """din_attention_top over the gather output rows [q (B) | k (B L)] (bf16, 16-B
    aligned rows): the rows' gradient comes back as one bf16 tensor.  The fused
    attention unit (one launch each way) when it covers the block."""
    L = his.shape[1]
    rows = _bf16_rows(rows)
    if DIN_FUSED and din_att_supported(rows.shape[1], att_mlp, att_out):
        w1, w2, w3 = (m.weight for m in _din_att_linears(att_mlp, att_out))
        b1, b2, b3 = (m.bias for m in _din_att_linears(att_mlp, att_out))
        return _DinAttFn.apply(rows, his, B, L, w1, b1, w2, b2, w3, b3)
    st = _DinState()
    feat = _DinRowsFeatFn.apply(rows, B, st, L)
    s = _din_scores(feat, att_mlp, att_out)
    r = rows.detach()
    return _DinPoolFn.apply(s, r[:B], r[B:], his, st, L)


def din_attention_top(q: torch.Tensor, k: torch.Tensor, his: torch.Tensor, att_mlp,
                      att_out: torch.nn.Linear) -> torch.Tensor:
    """The DIN top-MLP input [q | u] (bf16 [B, 2E]) on libmrec kernels: attention-unit
    input builder, MFMA attention MLP + Linear(h, 1), masked-softmax pooling; the
    backward is the pooling / builder kernels.  q [B, E], k [B*L, E] (bf16, the
    gathered target and history rows), his [B, L] ids (validity)."""
    B, E = q.shape
    L = his.shape[1]
    q, k = _bf16_rows(q), _bf16_rows(k)
    st = _DinState()
    feat = _DinFeatFn.apply(q, k, st, L)
    s = _din_scores(feat, att_mlp, att_out)
    return _DinPoolFn.apply(s, q, k, his, st, L)


def colsum(s: torch.Tensor, X: Optional[torch.Tensor], want_total: bool = True, *,
           out: Optional[torch.Tensor] = None, total: Optional[torch.Tensor] = None,
           sgd_lr: Optional[float] = None):
    """(sum_b s[b] X[b, :], sum_b s[b]) with libmrec's deterministic column sum.
    With ``sgd_lr`` the sums are applied in place as SGD to ``out`` / ``total``
    (parameters) instead: p -= lr * sum."""
    s = s.contiguous().float()
    C = 0 if X is None else X.shape[1]
    dev = s.device
    if out is None and C:
        out = torch.empty(C, dtype=torch.float32, device=dev)
    if total is None and want_total:
        total = torch.empty(1, dtype=torch.float32, device=dev)
    if X is not None and X.stride(1) != 1:
        X = X.contiguous()
    _mrec.call("mrec_colsum", s.data_ptr(), _mrec.ptr(X),
               _mrec.dtype_code(X.dtype) if X is not None else _mrec.F32,
               X.stride(0) if X is not None else 0, s.shape[0], C, _mrec.ptr(out),
               _mrec.ptr(total) if want_total else None, int(sgd_lr is not None),
               float(sgd_lr or 0.0), _mrec.stream_handle())
    return out, (total if want_total else None)


class _HeadFn(torch.autograd.Function):
    """z = base + h W^T + b for a Linear(H, 1) output layer (fp32 z [B])."""

    @staticmethod
    def forward(ctx, h, weight, bias, base, h_relu: bool):
        h = _bf16_rows(h)
        B, H = h.shape
        w = _weight_f32(weight).reshape(-1)
        b = bias.detach().float() if bias is not None else None
        base_c = base.detach().float().contiguous() if base is not None else None
        z = torch.empty(B, dtype=torch.float32, device=h.device)
        _mrec.call("mrec_head_fwd", h.data_ptr(), h.stride(0), B, H, w.data_ptr(), _mrec.ptr(b),
                   _mrec.ptr(base_c), z.data_ptr(), _mrec.stream_handle())
        ctx.save_for_backward(h, w)
        ctx.has_bias, ctx.has_base, ctx.h_relu = bias is not None, base is not None, h_relu
        ctx.weight, ctx.bias = weight, bias
        return z

    @staticmethod
    def backward(ctx, dz):
        h, w = ctx.saved_tensors
        B, H = h.shape
        dz = dz.contiguous().float()
        dh = None
        if ctx.needs_input_grad[0]:
            dh = _alloc(B, H, _BF16, dz.device)
            _mrec.call("mrec_head_bwd", dz.data_ptr(), w.data_ptr(), B, H,
                       h.data_ptr() if ctx.h_relu else None, h.stride(0), dh.data_ptr(),
                       dh.stride(0), _mrec.stream_handle())
            if ctx.h_relu:
                _stamp(dh, h)
        lr = sgd_lr(ctx.weight, ctx.bias)
        if lr is not None and ctx.weight.is_contiguous():
            colsum(dz, h, want_total=ctx.has_bias, out=ctx.weight.detach().view(-1),
                   total=ctx.bias.detach() if ctx.has_bias else None, sgd_lr=lr)
            dW = db = None
        else:
            dW, db = colsum(dz, h, want_total=ctx.has_bias)
            dW = dW.reshape(1, H)
        return dh, dW, db, (dz if ctx.has_base else None), None


def head(h: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
         base: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Logit of a Linear(H, 1) output layer plus an optional per-sample base logit
    (the FM / wide part): z = base + h W^T + b, fp32 [B]."""
    if not h.is_cuda:
        z = F.linear(h.float(), weight.float(), None if bias is None else bias.float()).reshape(-1)
        return z if base is None else z + base.float()
    return _HeadFn.apply(h, weight, bias, base, _is_relu_out(h))


# ----------------------------------------------------------------------------
# fused CTR head + BCE loss (the train step's last layer and its loss)
# ----------------------------------------------------------------------------

_TICKETS = {}
_ONES = {}


def _ticket(dev) -> torch.Tensor:
    t = _TICKETS.get(dev)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=dev)  # zero once; kernels leave it zero
        _TICKETS[dev] = t
    return t


def grad_one(dev) -> torch.Tensor:
    """Persistent scalar 1.0 used as the loss gradient (no fill kernel per step, and
    lets the fused head skip scaling its stashed gradients)."""
    t = _ONES.get(dev)
    if t is None:
        t = torch.ones((), dtype=torch.float32, device=dev)
        _ONES[dev] = t
    return t


class _CTRHeadBCEFn(torch.autograd.Function):
    """loss = BCEWithLogits(base + h W^T + b [+ xs ws + b2], y) (mean) for a
    Linear(H, 1) head (+ an optional side linear term: DeepFM's dense first-order
    weight and global bias).  The forward kernel also produces dh, dz and the
    parameter-gradient partials; the backward only reduces the partials (fused SGD
    of W, b, ws, b2 when compiled with plain SGD)."""

    @staticmethod
    def forward(ctx, h, weight, bias, base, ws, b2, y, xs, h_relu: bool):
        h = _bf16_rows(h)
        B, H = h.shape
        dev = h.device
        w = _weight_f32(weight).reshape(-1)
        b = bias.detach().float() if bias is not None else None
        base_c = base.detach().float().contiguous() if base is not None else None
        y = y.detach().float().contiguous()
        ns = 0
        if xs is not None:
            xs = xs.detach().float()
            if xs.stride(1) != 1:
                xs = xs.contiguous()
            ns = xs.shape[1]
        wsd = ws.detach().float().contiguous() if ws is not None else None
        b2d = b2.detach().float() if b2 is not None else None
        z = torch.empty(B, dtype=torch.float32, device=dev)
        dz = torch.empty(B, dtype=torch.float32, device=dev)
        dh = _alloc(B, H, _BF16, dev)
        nparts = int(_mrec.lib().mrec_ctr_head_parts(B))
        ldp = _r8(H + 1 + ns)
        part = torch.empty(nparts, ldp, dtype=torch.float32, device=dev)
        loss_part = torch.empty(nparts, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        _mrec.call("mrec_ctr_head_fwd", h.data_ptr(), h.stride(0), B, H, w.data_ptr(),
                   _mrec.ptr(b), _mrec.ptr(base_c), y.data_ptr(), _mrec.ptr(xs),
                   xs.stride(0) if xs is not None else 0, ns, _mrec.ptr(wsd), _mrec.ptr(b2d),
                   int(bool(h_relu)), z.data_ptr(), dz.data_ptr(), dh.data_ptr(), dh.stride(0),
                   part.data_ptr(), ldp, loss_part.data_ptr(), _ticket(dev).data_ptr(),
                   loss.data_ptr(), _mrec.stream_handle())
        if h_relu:
            _stamp(dh, h)
        ctx.save_for_backward(part, dz, dh)
        ctx.weight, ctx.bias, ctx.ws, ctx.b2 = weight, bias, ws, b2
        ctx.H, ctx.B, ctx.ns, ctx.has_base = H, B, ns, base is not None
        ctx.mark_non_differentiable(z)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for z
        return loss.reshape(()), z

    @staticmethod
    def backward(ctx, gloss, gz=None):
        part, dz, dh = ctx.saved_tensors
        dev = part.device
        g = gloss.detach().float().reshape(1).contiguous()
        one = g.data_ptr() == grad_one(dev).data_ptr()
        lr = sgd_lr(ctx.weight, ctx.bias, ctx.ws, ctx.b2)
        dW = db = dws = db2 = None
        det = (lambda t: None if t is None else t.detach())
        dpg = dp_grads(ctx.weight, ctx.bias, ctx.ws, ctx.b2) if lr is None else None
        if lr is not None and ctx.weight.is_contiguous():
            # independent of the backward GEMMs: rides along the next one
            defer_head_finish(_HeadFinish(part, ctx.B, ctx.H, ctx.ns, None if one else g, lr,
                                          ctx.weight.detach(), det(ctx.bias), det(ctx.ws),
                                          det(ctx.b2)))
        elif dpg is not None:
            defer_head_finish(_HeadFinish(part, ctx.B, ctx.H, ctx.ns, None if one else g, None,
                                          None, None, None, None, grads=dpg))
        else:
            f32 = dict(dtype=torch.float32, device=dev)
            dW = torch.empty(1, ctx.H, **f32)
            db = torch.empty(1, **f32) if ctx.bias is not None else None
            dws = torch.empty(ctx.ns, **f32) if ctx.ws is not None else None
            db2 = torch.empty(1, **f32) if ctx.b2 is not None else None
            _mrec.call("mrec_ctr_head_finish", part.data_ptr(), part.stride(0), ctx.B, ctx.H,
                       ctx.ns, g.data_ptr(), 0, 0.0, None, None, None, None, dW.data_ptr(),
                       _mrec.ptr(db), _mrec.ptr(dws), _mrec.ptr(db2), _mrec.stream_handle())
        if not one:
            dh = (dh.float() * g).to(_BF16)
            dz = dz * g
        return dh, dW, db, (dz if ctx.has_base else None), dws, db2, None, None, None


def ctr_head_bce(h: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                 base: Optional[torch.Tensor], y: torch.Tensor, xs: Optional[torch.Tensor] = None,
                 ws: Optional[torch.Tensor] = None, b2: Optional[torch.Tensor] = None):
    """(loss, z): mean BCE-with-logits of z = base + h W^T + b (+ xs ws + b2) against
    y — the CTR models' output layer and loss in one kernel (GPU, training) — else
    the plain ``head`` + torch loss."""
    ns = 0 if xs is None else xs.shape[1]
    if h.is_cuda and torch.is_grad_enabled() and h.shape[1] <= 1024 and ns <= 64:
        return _CTRHeadBCEFn.apply(h, weight, bias, base, ws, b2, y, xs, _is_relu_out(h))
    z = head(h, weight, bias, base)
    if xs is not None:
        z = z + xs.float() @ ws.float()
    if b2 is not None:
        z = z + b2.float()
    return F.binary_cross_entropy_with_logits(z.float(), y.float()), z


# ----------------------------------------------------------------------------
# fused MLP tower + CTR head + BCE (mrec_tower_fwd_bwd)
# ----------------------------------------------------------------------------

TOWER = os.environ.get("MREC_TOWER", "1") == "1"
TOWER_MAXL, TOWER_MAXW = 4, 512
# DCN-v2 cross layers inside the tower launch (MREC_TOWER_CROSS=0: the layered
# cross network of _CrossNetFn ahead of the tower)
TOWER_CROSS = os.environ.get("MREC_TOWER_CROSS", "1") == "1"
TOWER_MAXC = 3


def _mlp_linears(mlp) -> list:
    return [m.linear for m in mlp.mlp] if hasattr(mlp, "mlp") else list(mlp)


def tower_supported(x0: torch.Tensor, mlp, head: torch.nn.Linear, xs=None, cross=None) -> bool:
    """The fused tower covers the reference MLP (Linear -> ReLU per layer,
    Dense.py:4-24) with dropout 0 (or eval) + Linear(N_L, 1) + BCE on the GPU, and
    up to 3 DCN-v2 cross layers (``nn.Linear(d, d)``, d = the MLP's input width)
    ahead of it when the batch takes mrec_tower_dw."""
    if cross:
        lins = _mlp_linears(mlp) if (hasattr(mlp, "mlp") and mlp.mlp) else None
        if not TOWER_CROSS or not lins or len(cross) > TOWER_MAXC:
            return False
        d = lins[0].in_features
        if any(c.in_features != d or c.out_features != d or c.weight.dtype != torch.float32
               or not c.weight.is_contiguous() for c in cross):
            return False
        widths = [d] * len(cross) + [d] + [l.out_features for l in lins]
        if not _tdw_splits(x0.shape[0], widths):
            return False
    if not (TOWER and x0.is_cuda and torch.is_grad_enabled() and x0.dtype == _BF16):
        return False
    dense_layers = list(mlp.mlp) if hasattr(mlp, "mlp") else None
    if not dense_layers or len(dense_layers) > TOWER_MAXL:
        return False
    if any(d.dropout.p > 0 and d.training for d in dense_layers):
        return False
    lins = [d.linear for d in dense_layers]
    widths = [lins[0].in_features] + [l.out_features for l in lins]
    if any(w > TOWER_MAXW for w in widths) or head.out_features != 1:
        return False
    if any(l.weight.dtype != torch.float32 or not l.weight.is_contiguous() for l in lins):
        return False
    if xs is not None and xs.shape[1] > 64:
        return False
    return (x0.shape[1] >= widths[0] and x0.stride(1) == 1 and x0.stride(0) % 8 == 0
            and x0.data_ptr() % 16 == 0)


def _eff_split(K: int, s: int) -> int:
    """mrec_gemm's split-K count for K and a requested s (plan_split in gemm.hip)."""
    k = max(((K + s - 1) // s + 63) // 64 * 64, 64)
    return (K + k - 1) // k if K > 0 else 1


def _tdw_tiles(widths) -> int:
    """64 x 64 output tiles of the tower's dW_l = dY_l^T [X_l | 1]."""
    return sum(((widths[l + 1] + 63) // 64) * ((widths[l] + 1 + 63) // 64)
               for l in range(len(widths) - 1))


def _tdw_splits(B: int, widths=None) -> int:
    """K slices of mrec_tower_dw (0: not used): about 640 one-wave workgroups (2.5
    per CU) over the tiles, slices of >= 256 rows, at most 64 and at most B / 1024
    (but 4 allowed): the REDUCE that follows reads every slice's slab, and for a small
    tower it is the longer part.  4 for the C2 tower (147 tiles; 8 slices ran no
    faster and double the slabs the reduction reads) and for DIN's top tower (16
    tiles: 16 slices 0.2256-0.2258 ms/step, 8: 0.2245-0.2252, 4: 0.2233-0.2240), 64
    for DIN's layered attention unit (8 tiles over 204,800 rows)."""
    if os.environ.get("MREC_TOWER_DW", "1") == "0" or B < 256:
        return 0
    env = os.environ.get("MREC_TDW_SPLITS")  # A/B knob
    # at least 4 (C3's 245 tiles: 2 slices 0.1243 ms/step, 4: 0.1194; 3 and 5 slower,
    # tools/gpu_ab_splits.sh)
    want = int(env) if env else (4 if widths is None else
                                 max(4, min(64, 640 // _tdw_tiles(widths), max(4, B // 1024))))
    for s in range(want, 1, -1):
        if B // s >= 256 and _eff_split(B, s) == s:
            return s
    return 0


def _split_tower(widths, K: int) -> int:
    """K slices of the tower's weight-gradient GEMMs (generic mrec_gemm_multi path,
    dW_l [N_l, K_l + 1] over the batch), which share one launch: about two residency
    waves of 256-thread workgroups (3 per CU), slices of >= 256 rows."""
    tiles = sum(((widths[l + 1] + 63) // 64) * ((widths[l] + 1 + 63) // 64)
                for l in range(len(widths) - 1))
    s = 1
    while tiles * (s + 1) <= 640 and K // (s + 1) >= 256 and s < 64:
        s += 1
    return s


class _TowerBCEFn(torch.autograd.Function):
    """loss = BCEWithLogits(MLP(x0) . w + b + base [+ xs . ws + b2], y) (mean).
    Forward = ONE mrec_tower_fwd_bwd launch, which also produces every input /
    pre-activation gradient (dx0, dz, dh_l); backward = the weight-gradient GEMMs
    (one mrec_gemm_multi launch with the head finish; fused SGD when compiled with
    plain SGD, the split-K reductions ride in the next launch)."""

    @staticmethod
    def forward(ctx, x0, base, xs, y, n_layers, n_cross, *params):
        L, C = n_layers, n_cross
        Ws, bs = params[:L], params[L:2 * L]
        head_w, head_b, ws, b2 = params[2 * L:2 * L + 4]
        cWs, cbs = params[2 * L + 4:2 * L + 4 + C], params[2 * L + 4 + C:2 * L + 4 + 2 * C]
        B = x0.shape[0]
        dev = x0.device
        widths = [Ws[0].shape[1]] + [W.shape[0] for W in Ws]
        imgs = [tower_images(W) for W in Ws]
        cimgs = [tower_images(W) for W in cWs]
        # the weight gradients' operands: k-fragment images for mrec_tower_dw (the
        # tower writes them, x0's too), else row-major for the generic GEMM
        need_w = any(ctx.needs_input_grad[6:6 + 2 * L]) or any(
            ctx.needs_input_grad[6 + 2 * L + 4:6 + 2 * L + 4 + 2 * C])
        tdw = _tdw_splits(B, [widths[0]] * C + widths) if need_w else 0
        if C and need_w and not tdw:
            raise ValueError("cross layers in the tower need mrec_tower_dw (tower_supported)")
        cx_imgs, cdz_imgs = [], []
        if tdw:
            kf = lambda n: torch.empty(int(_mrec.lib().mrec_kfrag_elems(B, n)), dtype=_BF16,  # noqa: E731
                                       device=dev)
            hs = [kf(widths[l + 1]) for l in range(L - 1)]
            dhs = [kf(widths[l + 1]) for l in range(L)]
            x0_img = kf(widths[0])
            cx_imgs = [kf(widths[0]) for _ in range(C)]
            cdz_imgs = [kf(widths[0]) for _ in range(C)]
        else:
            hs = [_alloc(B, widths[l + 1], _BF16, dev) for l in range(L - 1)]
            dhs = [_alloc(B, widths[l + 1], _BF16, dev) for l in range(L)]
            x0_img = None
        dx0 = None
        if ctx.needs_input_grad[0]:  # x0's shape (it may carry zero pad columns past K0)
            Kx = x0.shape[1]
            dx0 = (_alloc(B, Kx, _BF16, dev) if _r8(Kx) == _r8(widths[0]) else
                   torch.zeros(B, _r8(Kx), dtype=_BF16, device=dev)[:, :Kx])
        dz = torch.empty(B, dtype=torch.float32, device=dev)
        ns = 0 if xs is None else xs.shape[1]
        if xs is not None:
            xs = xs.detach().float()
            if xs.stride(1) != 1:
                xs = xs.contiguous()
        H = widths[L]
        nparts = int(_mrec.lib().mrec_ctr_head_parts(B))
        ldp = _r8(H + 1 + ns)
        part = torch.empty(nparts, ldp, dtype=torch.float32, device=dev)
        loss_part = torch.empty(nparts, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        f32 = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
        hw, hb, wsd, b2d = f32(head_w).reshape(-1), f32(head_b), f32(ws), f32(b2)
        bsd = [f32(b) for b in bs]
        base_c = f32(base)
        yc = y.detach().float().contiguous()
        a = _mrec.TowerArgs()
        a.batch, a.n_layers = B, L
        for l in range(L + 1):
            a.width[l] = widths[l]
        a.x0, a.ld_x0 = x0.data_ptr(), x0.stride(0)
        for l in range(L):
            a.w_fwd[l], a.w_bwd[l] = imgs[l][0].data_ptr(), imgs[l][1].data_ptr()
            a.bias[l] = _mrec.ptr(bsd[l])
            a.dh_out[l], a.ld_dh[l] = dhs[l].data_ptr(), dhs[l].stride(0)
            if l < L - 1:
                a.h_out[l], a.ld_h[l] = hs[l].data_ptr(), hs[l].stride(0)
        a.kfrag, a.x0_img = int(bool(tdw)), _mrec.ptr(x0_img)
        cbsd = [f32(b) for b in cbs]
        a.n_cross = C
        for c in range(C):
            a.cross_w_fwd[c], a.cross_w_bwd[c] = cimgs[c][0].data_ptr(), cimgs[c][1].data_ptr()
            a.cross_bias[c] = _mrec.ptr(cbsd[c])
            if tdw:
                a.cross_x_img[c], a.cross_dz_img[c] = cx_imgs[c].data_ptr(), cdz_imgs[c].data_ptr()
        a.head_w, a.head_b, a.base = hw.data_ptr(), _mrec.ptr(hb), _mrec.ptr(base_c)
        a.xs, a.ld_xs, a.ns = _mrec.ptr(xs), xs.stride(0) if xs is not None else 0, ns
        a.ws, a.b2, a.y = _mrec.ptr(wsd), _mrec.ptr(b2d), yc.data_ptr()
        a.dx0, a.ld_dx0 = _mrec.ptr(dx0), dx0.stride(0) if dx0 is not None else 0
        a.z, a.dz = None, dz.data_ptr()
        a.part, a.ldp = part.data_ptr(), ldp
        a.loss_part, a.ticket, a.loss = loss_part.data_ptr(), _ticket(dev).data_ptr(), loss.data_ptr()
        with _timed("mrec_tower_fwd_bwd"):
            _mrec.call("mrec_tower_fwd_bwd", ctypes.byref(a), _mrec.stream_handle())
        ctx.save_for_backward(x0 if x0_img is None else x0_img, dz, part, dx0, *hs, *dhs, *cx_imgs,
                              *cdz_imgs)
        ctx.L, ctx.C, ctx.B, ctx.H, ctx.ns, ctx.widths = L, C, B, H, ns, widths
        ctx.tdw = tdw
        ctx.Ws, ctx.bs, ctx.imgs = Ws, bs, imgs
        ctx.cWs, ctx.cbs, ctx.cimgs = cWs, cbs, cimgs
        ctx.head = (head_w, head_b, ws, b2)
        ctx.has_base = base is not None
        ctx.mark_non_differentiable(dz)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, gloss):
        L, C, B = ctx.L, ctx.C, ctx.B
        saved = ctx.saved_tensors
        x0, dz, part, dx0 = saved[:4]
        hs, dhs = list(saved[4:4 + L - 1]), list(saved[4 + L - 1:4 + 2 * L - 1])
        cx_imgs = list(saved[4 + 2 * L - 1:4 + 2 * L - 1 + C]) if ctx.tdw else []
        cdz_imgs = list(saved[4 + 2 * L - 1 + C:]) if ctx.tdw else []
        dev = part.device
        g = gloss.detach().float().reshape(1).contiguous()
        one = g.data_ptr() == grad_one(dev).data_ptr()
        tdw = ctx.tdw
        if not one:  # a scaled loss: every stashed gradient scales with it
            dz = dz * g
            dx0 = (dx0.float() * g).to(_BF16) if dx0 is not None else None
            dhs = [(d.float() * g).to(_BF16) if tdw else _bf16_rows((d.float() * g).to(_BF16))
                   for d in dhs]
            cdz_imgs = [(d.float() * g).to(_BF16) for d in cdz_imgs]
        cross = None
        if C:  # cross layer c: dW = dz_c^T [x_c | 1]; the MLP's first X is x_C
            d = ctx.widths[0]
            cross = (ctx.cWs, ctx.cbs, ctx.cimgs, [(d, d)] * C, cdz_imgs, [x0] + cx_imgs[:-1])
            if tdw:
                x0 = cx_imgs[-1]
        need_w = any(ctx.needs_input_grad[6:6 + 2 * L]) or any(
            ctx.needs_input_grad[6 + 2 * L + 4:6 + 2 * L + 4 + 2 * C])
        grads = _tower_param_grads(ctx.widths, ctx.Ws, ctx.bs, ctx.imgs, ctx.head, B, ctx.H, ctx.ns,
                                   x0, hs, dhs, part, g, one, tdw, need_w, cross=cross)
        dWs, dbs, (dW_h, db_h, dws, db2), (cdWs, cdbs) = grads
        return (dx0, dz if ctx.has_base else None, None, None, None, None, *dWs, *dbs,
                dW_h, db_h, dws, db2, *cdWs, *cdbs)


def _tower_param_grads(widths, Ws, bs, imgs, head, B: int, H: int, ns: int, x0, hs, dhs, part, g,
                       one: bool, tdw: int, need_w: bool, cross=None):
    """The weight-gradient tail of a fused tower (BCE and given-dz modes): the L
    layers' dW = dh^T [h | 1] (mrec_tower_dw from the k-fragment images, else the
    generic split-K GEMMs) + the head parameters from the tower's partials; fused
    SGD / flat DP buffer / returned gradients as the parameters ask.  ``cross``
    (Ws, bs, imgs, dims, dys, xs): the cross layers ahead of the MLP, their dW =
    dz^T [x | 1] in the same mrec_tower_dw launch (tdw required).  ->
    (dWs, dbs, (dW_h, db_h, dws, db2), (cross dWs, cross dbs)), None where not
    returned."""
    head_w, head_b, ws, b2 = head
    L = len(Ws)
    dev = part.device
    xin = ([x0] if tdw else [x0[:, :widths[0]]]) + hs
    # every layer of the launch: (W, b, images, N, K, dY, X); cross layers first
    lay = []
    if cross is not None:
        cW, cb, cim, cdims, cdy, cx = cross
        lay += [(cW[c], cb[c], cim[c], cdims[c][0], cdims[c][1], cdy[c] if tdw else None,
                 cx[c] if tdw else None) for c in range(len(cW))]
    C = len(lay)
    lay += [(Ws[l], bs[l], imgs[l], widths[l + 1], widths[l], dhs[l], xin[l]) for l in range(L)]
    # --- weight gradients of the layers: one launch ---
    lr = sgd_lr(*[t[0] for t in lay], *[t[1] for t in lay])
    dpg = dp_grads(*[t[0] for t in lay], *[t[1] for t in lay]) if lr is None else None
    n = len(lay)
    dWs, dbs = [None] * n, [None] * n
    calls = []
    if need_w:
        sk = tdw or _split_tower(widths, B)
        ph = _mrec.GEMM_PARTIAL if sk > 1 else _mrec.GEMM_FULL
        # with mrec_tower_dw the calls below only carry the REDUCE phase's
        # arguments (its operands are never read: k-fragment images as stand-ins)
        opnd = (lambda t: t.view(-1, 8)) if tdw else (lambda t: t)  # noqa: E731
        for i, (W, bias_l, img, N, K, dy, xx) in enumerate(lay):
            if lr is not None:
                c = _Call(opnd(dy), _mrec.LAYOUT_COL, opnd(xx), _mrec.LAYOUT_COL, N, K, B, ph,
                          ones_out=bias_l.detach() if bias_l is not None else None,
                          out=W.detach(), out_dtype=torch.float32, split_k=sk, sgd_lr=lr,
                          img_row=img[0], img_tr=img[1], img_kind=_mrec.IMG_TOWER)
                images_updated(W, "tower")
            elif dpg is not None:
                c = _Call(opnd(dy), _mrec.LAYOUT_COL, opnd(xx), _mrec.LAYOUT_COL, N, K, B, ph,
                          ones_out=dpg[n + i], out=dpg[i], out_dtype=torch.float32,
                          split_k=sk)
            else:
                dWs[i] = torch.empty(N, K, dtype=torch.float32, device=dev)
                dbs[i] = (torch.empty(N, dtype=torch.float32, device=dev)
                          if bias_l is not None else None)
                c = _Call(opnd(dy), _mrec.LAYOUT_COL, opnd(xx), _mrec.LAYOUT_COL, N, K, B, ph,
                          ones_out=dbs[i], out=dWs[i], out_dtype=torch.float32, split_k=sk)
            calls.append(c)
    # --- the head's parameters (w, b, ws, b2): fixed-order partial sums ---
    hlr = sgd_lr(head_w, head_b, ws, b2)
    det = (lambda t: None if t is None else t.detach())
    hdp = dp_grads(head_w, head_b, ws, b2) if hlr is None else None
    dW_h = db_h = dws = db2 = None
    if hlr is not None and head_w.is_contiguous():
        defer_head_finish(_HeadFinish(part, B, H, ns, None if one else g, hlr,
                                      head_w.detach(), det(head_b), det(ws), det(b2)))
    elif hdp is not None:
        defer_head_finish(_HeadFinish(part, B, H, ns, None if one else g, None,
                                      None, None, None, None, grads=hdp))
    else:
        f32 = dict(dtype=torch.float32, device=dev)
        dW_h = torch.empty(1, H, **f32)
        db_h = torch.empty(1, **f32) if head_b is not None else None
        dws = torch.empty(ns, **f32) if ws is not None else None
        db2 = torch.empty(1, **f32) if b2 is not None else None
        _mrec.call("mrec_ctr_head_finish", part.data_ptr(), part.stride(0), B, H, ns,
                   g.data_ptr(), 0, 0.0, None, None, None, None, dW_h.data_ptr(),
                   _mrec.ptr(db_h), _mrec.ptr(dws), _mrec.ptr(db2), _mrec.stream_handle())
    if calls and tdw:
        _tower_dw(calls, [t[5] for t in lay], [t[6] for t in lay], [(t[3], t[4]) for t in lay], B,
                  tdw)
        if lr is None and dpg is None:
            _run_all([c.with_phase(_mrec.GEMM_REDUCE) for c in calls])
        else:
            for c in calls:
                _defer(c)
    elif calls:
        launch_multi(calls)
        if calls[0].args[8] > 1:  # split-K partial slabs: now the reductions
            if lr is None and dpg is None:
                # returned gradients: autograd may copy them on return, so they must
                # be complete before this backward returns
                _run_all([c.with_phase(_mrec.GEMM_REDUCE) for c in calls])
            else:  # in-place SGD / flat DP buffer: ride in the next launches
                for c in calls:
                    _defer(c)
    else:
        _flush_finish()
    return dWs[C:], dbs[C:], (dW_h, db_h, dws, db2), (dWs[:C], dbs[:C])


def _run_all(jobs):
    for i in range(0, len(jobs), 4):
        _run(jobs[i:i + 4])


def _tower_dw(calls, dys, xins, dims, B: int, splits: int):
    """The tower's weight-gradient partial slabs by mrec_tower_dw from the
    k-fragment images (+ the deferred CTR head finish in the same launch); the
    split-K REDUCE of each call (fused SGD / flat DP buffer / returned gradient)
    follows as usual.  Pending reductions that write what this reads run first."""
    global _PENDING
    reads = {t.data_ptr() for t in list(dys) + list(xins)}
    if any(p.writes & reads for p in _PENDING):
        _run_all(_PENDING)
        _PENDING = []
    a = _mrec.TowerDwArgs()
    a.n_layers, a.batch, a.splits = len(calls), B, splits
    for l, c in enumerate(calls):
        a.n_out[l], a.n_in[l] = dims[l]
        a.dy_img[l], a.x_img[l] = dys[l].data_ptr(), xins[l].data_ptr()
        a.ws[l], a.ldws[l] = c.ws.data_ptr(), (dims[l][1] + 1 + 7) // 8 * 8
    fin = _FINISH.pop(0) if _FINISH else None
    feed = take_feed_job()
    with _timed("mrec_tower_dw"):
        _mrec.call("mrec_tower_dw_ex", ctypes.byref(a), ctypes.byref(fin.struct) if fin else None,
                   ctypes.byref(feed) if feed is not None else None, _mrec.stream_handle())
    pend = _PENDING
    _PENDING = []
    _run_all(pend)


def tower_bce(x0: torch.Tensor, mlp, head: torch.nn.Linear, base: Optional[torch.Tensor],
              y: torch.Tensor, xs: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
              b2: Optional[torch.Tensor] = None, cross=None) -> torch.Tensor:
    """Training loss of a CTR model's deep part: mean BCE-with-logits of
    MLP(x0) . head.weight + head.bias + base (+ xs . ws + b2) — the reference MLP
    (MLP.py:8-23) and Linear(N_L, 1) — as one fused tower launch (caller checks
    ``tower_supported``).  ``cross``: DCN-v2 cross layers (``nn.Linear(d, d)``)
    applied to x0 ahead of the MLP in the same launch (mrec_tower_args.n_cross)."""
    lins = _mlp_linears(mlp)
    cross = list(cross or [])
    params = ([l.weight for l in lins] + [l.bias for l in lins] +
              [head.weight, head.bias, ws, b2] + [c.weight for c in cross] + [c.bias for c in cross])
    return _TowerBCEFn.apply(x0, base, xs, y, len(lins), len(cross), *params)


class _ScoreTowerFn(torch.autograd.Function):
    """s = MLP(x0) . w + b per row (fp32 [B]): DIN's attention unit (att_mlp +
    att_out over the [q, k, q-k, q*k] rows) on the fused tower.  Forward = one
    MREC_TOWER_FORWARD launch (the scores only, nothing else leaves LDS); backward =
    one MREC_TOWER_GIVEN_DZ launch with dz = ds (the forward recomputed in LDS:
    dx0 and every pre-activation gradient, the k-fragment images) + mrec_tower_dw +
    the head finish, as the BCE tower's backward."""

    @staticmethod
    def _args(x0, widths, imgs, bsd, hw, hb):
        a = _mrec.TowerArgs()
        L = len(widths) - 1
        a.batch, a.n_layers = x0.shape[0], L
        for l in range(L + 1):
            a.width[l] = widths[l]
        a.x0, a.ld_x0 = x0.data_ptr(), x0.stride(0)
        for l in range(L):
            a.w_fwd[l], a.w_bwd[l] = imgs[l][0].data_ptr(), imgs[l][1].data_ptr()
            a.bias[l] = _mrec.ptr(bsd[l])
        a.head_w, a.head_b = hw.data_ptr(), _mrec.ptr(hb)
        return a

    @staticmethod
    def forward(ctx, x0, n_layers, *params):
        L = n_layers
        Ws, bs = params[:L], params[L:2 * L]
        head_w, head_b = params[2 * L:2 * L + 2]
        B = x0.shape[0]
        widths = [Ws[0].shape[1]] + [W.shape[0] for W in Ws]
        imgs = [tower_images(W) for W in Ws]
        f32 = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
        bsd, hw, hb = [f32(b) for b in bs], f32(head_w).reshape(-1), f32(head_b)
        z = torch.empty(B, dtype=torch.float32, device=x0.device)
        a = _ScoreTowerFn._args(x0, widths, imgs, bsd, hw, hb)
        a.mode, a.z, a.ldp = _mrec.TOWER_FORWARD, z.data_ptr(), _r8(widths[L] + 1)
        _mrec.call("mrec_tower_fwd_bwd", ctypes.byref(a), _mrec.stream_handle())
        ctx.save_for_backward(x0)
        ctx.L, ctx.widths, ctx.Ws, ctx.bs, ctx.imgs = L, widths, Ws, bs, imgs
        ctx.head = (head_w, head_b, None, None)
        ctx.keep = (bsd, hw, hb)
        return z

    @staticmethod
    def backward(ctx, ds):
        x0, = ctx.saved_tensors
        L, widths = ctx.L, ctx.widths
        B = x0.shape[0]
        dev = x0.device
        ds = ds.detach().float().reshape(B).contiguous()
        need_w = any(ctx.needs_input_grad[2:2 + 2 * L])
        tdw = _tdw_splits(B, widths) if need_w else 0
        if tdw:
            kf = lambda n: torch.empty(int(_mrec.lib().mrec_kfrag_elems(B, n)), dtype=_BF16,  # noqa: E731
                                       device=dev)
            hs = [kf(widths[l + 1]) for l in range(L - 1)]
            dhs = [kf(widths[l + 1]) for l in range(L)]
            x0_img = kf(widths[0])
        else:
            hs = [_alloc(B, widths[l + 1], _BF16, dev) for l in range(L - 1)]
            dhs = [_alloc(B, widths[l + 1], _BF16, dev) for l in range(L)]
            x0_img = None
        dx0 = None
        if ctx.needs_input_grad[0]:
            Kx = x0.shape[1]
            dx0 = (_alloc(B, Kx, _BF16, dev) if _r8(Kx) == _r8(widths[0]) else
                   torch.zeros(B, _r8(Kx), dtype=_BF16, device=dev)[:, :Kx])
        H = widths[L]
        ldp = _r8(H + 1)
        part = torch.empty(int(_mrec.lib().mrec_ctr_head_parts(B)), ldp, dtype=torch.float32,
                           device=dev)
        bsd, hw, hb = ctx.keep
        a = _ScoreTowerFn._args(x0, widths, ctx.imgs, bsd, hw, hb)
        for l in range(L):
            a.dh_out[l], a.ld_dh[l] = dhs[l].data_ptr(), dhs[l].stride(0)
            if l < L - 1:
                a.h_out[l], a.ld_h[l] = hs[l].data_ptr(), hs[l].stride(0)
        a.kfrag, a.x0_img = int(bool(tdw)), _mrec.ptr(x0_img)
        a.dx0, a.ld_dx0 = _mrec.ptr(dx0), dx0.stride(0) if dx0 is not None else 0
        a.part, a.ldp = part.data_ptr(), ldp
        a.mode, a.dz_in = _mrec.TOWER_GIVEN_DZ, ds.data_ptr()
        _mrec.call("mrec_tower_fwd_bwd", ctypes.byref(a), _mrec.stream_handle())
        g = grad_one(dev)
        dWs, dbs, (dW_h, db_h, _, _), _ = _tower_param_grads(
            widths, ctx.Ws, ctx.bs, ctx.imgs, ctx.head, B, H, 0, x0_img if tdw else x0, hs, dhs,
            part, g, True, tdw, need_w)
        return (dx0, None, *dWs, *dbs, dW_h, db_h)


def score_tower(x0: torch.Tensor, mlp, head: torch.nn.Linear) -> torch.Tensor:
    """MLP(x0) . head.weight + head.bias per row (fp32 [B]) on the fused tower
    (caller checks ``tower_supported``): DIN's attention-unit scores."""
    lins = _mlp_linears(mlp)
    params = [l.weight for l in lins] + [l.bias for l in lins] + [head.weight, head.bias]
    return _ScoreTowerFn.apply(x0, len(lins), *params)
