"""Microbenchmark of the embedding-backward plan kernel on the C2 bank
(26 x 38462 rows, batch 4096), optionally with per-phase wall-clock stamps
from a library built with -DMREC_PLAN_PROF (MREC_LIB_PATH=...)."""
import ctypes
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchrec_amd import _mrec  # noqa: E402
from pytorchrec_amd.embedding import EmbeddingBank  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 38462
    bank = EmbeddingBank([rows] * 26, 16, with_first_order=True, dtype=torch.bfloat16,
                         update="sgd", device="cuda")
    zipf = len(sys.argv) > 3 and sys.argv[3] == "zipf"
    if zipf:
        import numpy as np
        z = np.minimum(np.random.default_rng(0).zipf(1.05, (B, 26)) - 1, rows - 1)
        ids2 = torch.from_numpy(z.astype(np.int32)).cuda()
    else:
        ids2 = torch.randint(0, rows, (B, 26), dtype=torch.int32, device="cuda")
    if len(sys.argv) > 4 and sys.argv[4] == "cols":  # per-field [B] columns (bench.py's layout)
        cols = [ids2[:, f].contiguous() for f in range(26)]
        idd = _mrec.IdsDesc(cols)
    else:
        idd = _mrec.IdsDesc(None, stacked=ids2)  # [B, 26] int32
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(26, B)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")

    def _plan():
        _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), idd.ref(), B, ws.data_ptr(), wsb,
                   None, bank.step_counter().data_ptr(), _mrec.stream_handle())
    for _ in range(10):
        _plan()
    torch.cuda.synchronize()
    n = 200
    # graph-captured back-to-back launches: device time, no host launch overhead
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                _plan()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    print(f"plan B={B} rows={rows} zipf={zipf}: {e0.elapsed_time(e1) * 1e3 / n:.2f} us/launch")
    lib = _mrec.lib()
    if hasattr(lib, "mrec_plan_prof_read"):
        buf = (ctypes.c_uint64 * 16)()
        lib.mrec_plan_prof_read(buf)
        t = [buf[i] for i in range(16)]
        print("phase ns (100 MHz wall clock):", [(t[i + 1] - t[i]) * 10 for i in range(4)],
              "total", (t[4] - t[0]) * 10)
        print("sort passes / segments ns:", [(t[i] - t[3]) * 10 for i in range(5, 10)])


if __name__ == "__main__":
    main()
