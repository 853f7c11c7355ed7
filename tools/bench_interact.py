"""Time the C2 interaction launch (mrec_interact_fwd: 26 x 38,462-row bf16 bank,
D = 16 + first-order column, B = 4096, x0 bf16 [B, 432]) and, with a library built
with -DMREC_INTERACT_PROF (MREC_LIB_PATH=...), print the per-sample phase stamps of
one launch: start, first id landed, rows landed, sums done, end (us after the
earliest start; min / median / max over the samples)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchrec_amd import _mrec  # noqa: E402
from pytorchrec_amd.embedding import EmbeddingBank, interact  # noqa: E402


def main():
    B, F, rows = 4096, 26, 38462
    dev = torch.device("cuda")
    bank = EmbeddingBank([rows] * F, 16, with_first_order=True, dtype=torch.bfloat16, device=dev)
    with torch.no_grad():
        bank.weight.normal_(0, 0.01)
    bank.check_ids = False  # no OOB flag read-back (graph capture)
    ids = torch.randint(0, rows, (F, B), dtype=torch.int32, device=dev)
    idl = [ids[f] for f in range(F)]  # per-field columns, as the models pass them
    dense = torch.rand(B, 13, device=dev)
    dw = torch.randn(13, device=dev) * 0.1
    bias = torch.zeros(1, device=dev)

    def run():
        with torch.no_grad():
            return interact(bank, idl, dense, dw, bias, fm2=True, first_order=True, x0_cols=432,
                            x0_dtype=torch.bfloat16)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    n = 100
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                run()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    print(f"interact B={B}: {e0.elapsed_time(e1) * 1e3 / n:.2f} us/launch")
    lib = _mrec.lib()
    if not hasattr(lib, "mrec_interact_prof_read"):
        return
    run()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (5 * B))()
    lib.mrec_interact_prof_read(buf, B)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(B, 5).astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) * 0.01
    for k, name in enumerate(["start", "id landed", "rows landed", "sums done", "end"]):
        c = us[:, k]
        print(f"{name:>12}: min {c.min():6.2f} med {np.median(c):6.2f} p90 {np.percentile(c, 90):6.2f} "
              f"max {c.max():6.2f} us")
    d = np.diff(us, axis=1)
    for k, name in enumerate(["id latency", "row latency", "sums", "dense+stores"]):
        print(f"{name:>12}: med {np.median(d[:, k]):6.2f} p90 {np.percentile(d[:, k], 90):6.2f} us")


if __name__ == "__main__":
    main()
