"""Microbenchmark of the embedding-backward apply kernel on the C2 bank
(26 x 38462 rows, D=16 bf16 + first-order weight, batch 4096, DeepFM inputs:
dx, FM2 terms and first-order grads).  MREC_LIB_PATH selects a library variant."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchrec_amd import _mrec  # noqa: E402
from pytorchrec_amd.embedding import EmbeddingBank  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    rows, F, D = 38462, 26, 16
    bank = EmbeddingBank([rows] * F, D, with_first_order=True, dtype=torch.bfloat16,
                         update="sgd", device="cuda")
    ids2 = torch.randint(0, rows, (B, F), dtype=torch.int32, device="cuda")
    idd = _mrec.IdsDesc(None, stacked=ids2)
    wsb = _mrec.lib().mrec_emb_bwd_workspace_size(F, B)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    _mrec.call("mrec_emb_bwd_plan", bank.desc().ref(), idd.ref(), B, ws.data_ptr(), wsb,
               None, bank.step_counter().data_ptr(), _mrec.stream_handle())
    dx = (torch.randn(B, 448, device="cuda") * 1e-3).to(torch.bfloat16)
    x0 = torch.randn(B, 448, device="cuda").to(torch.bfloat16)
    dfm = torch.randn(B, device="cuda") * 1e-3
    fm_sum = torch.randn(B, D, device="cuda")
    dw = torch.randn(B, device="cuda") * 1e-3

    def apply():
        _mrec.call("mrec_emb_bwd_apply", bank.desc().ref(), B, ws.data_ptr(), wsb,
                   dx.data_ptr(), _mrec.BF16, 448, dfm.data_ptr(), fm_sum.data_ptr(),
                   x0.data_ptr(), _mrec.BF16, 448, dw.data_ptr(), _mrec.BWD_SGD, 0.01,
                   1234, bank.step_counter().data_ptr(), None, _mrec.stream_handle())

    for _ in range(10):
        apply()
    torch.cuda.synchronize()
    n = 200
    # graph-captured back-to-back launches: device time, no host launch overhead
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                apply()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    print(f"apply B={B} {_mrec.LIB_PATH.rsplit('/', 1)[-1]}: {e0.elapsed_time(e1) * 1e3 / n:.2f} us/launch")


if __name__ == "__main__":
    main()
