"""Microbenchmark of libmrec's MFMA GEMM on the DeepFM MLP shapes (B = 4096).

    python tools/bench_gemm.py [--reps 200] [--only fwd|dx|dw]

Prints per-shape average kernel time (HIP events around back-to-back launches on
one stream, graph-captured to strip host overhead) and, for reference, torch's
own matmul (hipBLASLt) on the same shape.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorchrec_amd import _mrec, dense as D  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps // 10):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps // 10 * 10)


def prof_report(fn):
    import ctypes
    import numpy as np
    n = 4096
    buf = (ctypes.c_uint64 * (4 * n))()
    _mrec.lib().mrec_gemm_prof_read(buf, n)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
    t = t[(t[:, 0] > 0) & (t[:, 3] >= t[:, 0])]
    recent = t[:, 0] >= t[:, 0].max() - 100000  # the last launch only (1 ms window)
    t = t[recent]
    t0 = t[:, 0].min()
    ns = lambda x: x * 10  # noqa: E731
    q = lambda x: np.percentile(ns(x), [0, 50, 100]).round(0).tolist()  # noqa: E731
    print(f"    {len(t)} workgroups; span {ns(t[:, 3].max() - t0)} ns")
    print(f"    start offset  min/med/max {q(t[:, 0] - t0)}")
    print(f"    first group   {q(t[:, 1] - t[:, 0])}")
    print(f"    main loop     {q(t[:, 2] - t[:, 1])}")
    print(f"    epilogue      {q(t[:, 3] - t[:, 2])}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--only", default="")
    ap.add_argument("--prof", action="store_true",
                    help="print per-workgroup phase times (library built with -DMREC_GEMM_PROF)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, N, K = 4096, 400, 429
    x = D._alloc(M, 432, torch.bfloat16, dev)
    x.normal_()
    W = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev) * 0.05
    wr, wt = D.weight_prep(W)
    y = D._alloc(M, N, torch.bfloat16, dev)
    y.normal_()
    dy = D._alloc(M, N, torch.bfloat16, dev)
    dy.normal_()
    dW = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    flop = 2 * M * N * K
    cases = {
        "fwd": lambda: D.gemm(x, _mrec.LAYOUT_ROW, wr[:, :K], _mrec.LAYOUT_ROW, M, N, K, bias=b,
                              act=_mrec.ACT_RELU, out=y),
        "dx": lambda: D.gemm(dy, _mrec.LAYOUT_ROW, wt, _mrec.LAYOUT_ROW, M, 432, N, b_cols=K,
                             mask=x),
        "dw": lambda: D.gemm(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M, ones_out=db,
                             out=dW),
        "prep": lambda: D.weight_prep(W),
    }
    xb = x[:, :K].contiguous()
    wb = W.to(torch.bfloat16)
    dyb = dy.contiguous()
    ref = {
        "fwd": lambda: torch.nn.functional.linear(xb, wb),
        "dx": lambda: dyb @ wb,
        "dw": lambda: dyb.t() @ xb,
    }
    tiny = torch.zeros(1, device=dev)
    cases["empty-kernel"] = lambda: tiny.add_(1.0)
    for kk in (64, 128, 256):
        xk = D._alloc(M, kk, torch.bfloat16, dev)
        xk.normal_()
        wk, _ = D.weight_prep(torch.randn(N, kk, device=dev) * 0.05)
        cases[f"fwd/K{kk}"] = (lambda xk=xk, wk=wk, kk=kk: D.gemm(xk, _mrec.LAYOUT_ROW, wk[:, :kk],
                                                                 _mrec.LAYOUT_ROW, M, N, kk))
    for sk in (1, 2, 4, 8):
        cases[f"dw/s{sk}"] = (lambda sk=sk: D.gemm(dy, _mrec.LAYOUT_COL, x, _mrec.LAYOUT_COL, N, K, M,
                                                   ones_out=db, out=dW, split_k=sk))
    # the tower's three weight-gradient GEMMs as ONE mrec_gemm_multi launch (PARTIAL
    # phase, as in the training step; split from dense._split_tower)
    widths = [429, 400, 400, 400]
    sk3 = D._split_tower(widths, M)
    xs3 = [x] + [D._alloc(M, 400, torch.bfloat16, dev).normal_() for _ in range(2)]
    dys3 = [D._alloc(M, 400, torch.bfloat16, dev).normal_() for _ in range(3)]
    calls3 = [D._Call(dys3[l], _mrec.LAYOUT_COL, xs3[l][:, :widths[l]], _mrec.LAYOUT_COL, 400,
                      widths[l], M, _mrec.GEMM_PARTIAL if sk3 > 1 else _mrec.GEMM_FULL,
                      ones_out=torch.empty(400, device=dev), out_dtype=torch.float32, split_k=sk3)
              for l in range(3)]
    print(f"dw3: split_k {sk3}")
    cases["dw3"] = lambda: D._run(calls3)
    # the same three weight gradients by mrec_tower_dw on k-fragment images
    import ctypes
    lib = _mrec.lib()
    for ksplit in (4, 5, 8):
        ta = _mrec.TowerDwArgs()
        ta.n_layers, ta.batch, ta.splits = 3, M, ksplit
        keep = []
        for l in range(3):
            ims = []
            for t, n in ((dys3[l], 400), (xs3[l], widths[l])):
                im = torch.zeros(int(lib.mrec_kfrag_elems(M, n)), dtype=torch.bfloat16, device=dev)
                _mrec.call("mrec_kfrag_pack", t.data_ptr(), M, n, t.stride(0), im.data_ptr(),
                           _mrec.stream_handle())
                ims.append(im)
            wsb = int(lib.mrec_gemm_workspace_size(400, widths[l], M, ksplit))
            ws = torch.empty(wsb // 4, dtype=torch.float32, device=dev)
            keep += ims + [ws]
            ta.n_out[l], ta.n_in[l] = 400, widths[l]
            ta.dy_img[l], ta.x_img[l] = ims[0].data_ptr(), ims[1].data_ptr()
            ta.ws[l], ta.ldws[l] = ws.data_ptr(), (widths[l] + 1 + 7) // 8 * 8
        cases[f"tdw/s{ksplit}"] = (lambda ta=ta, keep=keep: _mrec.call(
            "mrec_tower_dw", ctypes.byref(ta), None, _mrec.stream_handle()))
    for name, fn in cases.items():
        if a.only and not name.startswith(a.only):
            continue
        t = timed(fn, a.reps)
        line = f"{name:5s} mrec {t:8.2f} us  {flop / t / 1e6:8.1f} TFLOP/s"
        if name in ref:
            tr = timed(ref[name], a.reps)
            line += f"   | torch/hipBLASLt {tr:8.2f} us"
        print(line, flush=True)
        if a.prof and hasattr(_mrec.lib(), "mrec_gemm_prof_read"):
            fn()
            torch.cuda.synchronize()
            prof_report(fn)


if __name__ == "__main__":
    main()
