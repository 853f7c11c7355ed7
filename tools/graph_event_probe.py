"""Can a kernel INSIDE a replayed HIP graph be timed with events?  torch's
``Event(external=True)`` records become event-record nodes of the captured graph
(cudaEventRecordExternal semantics).  Captures [a | b | c] with external timing
events around b, replays it, and prints the per-replay event interval next to b's
duration when b runs alone -- run under rocprofv3 --kernel-trace --stats to compare
with the profiler's in-graph duration of b.  (the roofline must
be the in-step figure.)"""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    z = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    big = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    e0 = torch.cuda.Event(enable_timing=True, external=True)
    e1 = torch.cuda.Event(enable_timing=True, external=True)

    def body(timed):
        big.fill_(1.0)                      # a
        if timed:
            e0.record()
        torch.mm(x, y, out=z)               # b (the timed kernel)
        if timed:
            e1.record()
        big.mul_(0.5)                       # c

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(False)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(True)
    ins = []
    for _ in range(30):
        g.replay()
        torch.cuda.synchronize()
        ins.append(e0.elapsed_time(e1) * 1e3)
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
