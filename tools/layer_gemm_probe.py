"""How fast can ONE layer of the C2 tower run as its own GEMM launch on MI355X?
(Design probe for the layered-vs-fused tower question)  Times the
tower's layer shapes with torch.mm (hipBLASLt / rocBLAS) inside a replayed HIP graph,
each GEMM between two others so launch gaps are the in-graph ones:

  fwd   [4096, 432] x [432, 400], [4096, 400] x [400, 400]
  dx    [4096, 400] x [400, 432], [4096, 400] x [400, 400]
  dW    [400, 4096] x [4096, 432]

Run under rocprofv3 --kernel-trace --stats for per-kernel durations."""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    M = 4096
    shapes = {"fwd1": (M, 432, 400), "fwd2": (M, 400, 400), "dx1": (M, 400, 432),
              "dx2": (M, 400, 400), "dw1": (400, M, 432)}
    ops = {}
    for k, (m, kk, n) in shapes.items():
        a = torch.randn(m, kk, device=dev, dtype=bf)
        b = torch.randn(kk, n, device=dev, dtype=bf)
        c = torch.empty(m, n, device=dev, dtype=bf)
        ops[k] = (a, b, c)

    def body():
        for k, (a, b, c) in ops.items():
            torch.mm(a, b, out=c)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(4):
            body()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 50
    for _ in range(n):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) * 1e3 / (n * 4)
    print(json.dumps({"us_per_body_of_5_gemms": round(per, 2),
                      "flop": {k: 2 * m * kk * nn for k, (m, kk, nn) in shapes.items()}}))


if __name__ == "__main__":
    main()
