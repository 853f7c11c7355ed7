"""Batch sweep of the fused interaction kernel (mrec_interact_fwd, no plan):
device time per launch (graph-captured back-to-back launches) and algorithmic
GB/s (DESIGN.md §3 bytes/sample) at B = 64 .. 262144, on a C2-sized bank
(26 x 38,462 rows, MALL-resident) and a 26 x 4M-row bank (6.6 GB, HBM-resident).
Separates the per-launch latency floor from the bandwidth term."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchrec_amd import _mrec  # noqa: E402
from pytorchrec_amd.embedding import EmbeddingBank, init_bank_  # noqa: E402

F, D, ND, X0 = 26, 16, 13, 432


def time_graph(fn, n=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda")
    for rows in (38462, 4_000_000):
        bank = EmbeddingBank([rows] * F, D, with_first_order=True, dtype=torch.bfloat16,
                             update="sgd", device=dev)
        init_bank_(bank, generator=torch.Generator(device=dev).manual_seed(1))
        for B in (64, 1024, 4096, 16384, 65536, 262144):
            ids2 = torch.randint(0, rows, (F, B), dtype=torch.int32, device=dev)
            idd = _mrec.IdsDesc([ids2[f] for f in range(F)])
            dense = torch.rand(B, ND, device=dev)
            dw = torch.randn(ND, device=dev)
            bias = torch.zeros(1, device=dev)
            x0 = torch.empty(B, X0, dtype=torch.bfloat16, device=dev)
            logit = torch.empty(B, device=dev)
            fm = torch.empty(B, D, device=dev)

            def fwd():
                _mrec.call("mrec_interact_fwd", bank.desc().ref(), idd.ref(), B, dense.data_ptr(),
                           ND, ND, dw.data_ptr(), bias.data_ptr(), 3, x0.data_ptr(), _mrec.BF16,
                           X0, X0, logit.data_ptr(), fm.data_ptr(), None, _mrec.stream_handle())
            us = time_graph(fwd)
            nbytes = B * (F * 4 + F * (D + 1) * 2 + ND * 4 + X0 * 2 + 4 + D * 4)
            print(f"interact rows={rows:>8} B={B:>7}: {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s",
                  flush=True)
        del bank
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
