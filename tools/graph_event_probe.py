"""Can a kernel INSIDE a replayed HIP graph be timed with events?  bench.py's
GraphKernelTimer splices event-record nodes around chosen kernel nodes of a
captured graph (torch refuses Event(external=True) on ROCm).  Captures [a | b | c],
times b inside the replayed graph, and prints it next to b's duration when b runs
alone -- run under rocprofv3 --kernel-trace --stats to compare with the profiler's
in-graph duration of b.  (the roofline must be the in-step
figure.)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import GraphKernelTimer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    z = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    big = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    timer = GraphKernelTimer()

    def body(timed):
        big.fill_(1.0)                      # a
        if timed:
            timer.begin()
        torch.mm(x, y, out=z)               # b (the timed kernel)
        if timed:
            timer.end("mm")
        big.mul_(0.5)                       # c

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(False)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        body(True)
    timer.arm(g.raw_cuda_graph())
    g.instantiate()
    ins = []
    for _ in range(30):
        g.replay()
        torch.cuda.synchronize()
        ins.append(timer.elapsed(0) * 1e6)
    a0 = torch.cuda.Event(enable_timing=True)
    a1 = torch.cuda.Event(enable_timing=True)
    alone = []
    for _ in range(30):
        a0.record()
        torch.mm(x, y, out=z)
        a1.record()
        torch.cuda.synchronize()
        alone.append(a0.elapsed_time(a1) * 1e3)
    ins.sort()
    alone.sort()
    print(json.dumps({"in_graph_us_median": ins[len(ins) // 2], "in_graph_us_min": ins[0],
                      "eager_alone_us_median": alone[len(alone) // 2],
                      "gemm_flop": 2 * 4096 ** 3}))


if __name__ == "__main__":
    main()
