"""Do two independent kernels captured on two streams of one HIP graph run at the
same time?  Two ~N us spin kernels (torch.cuda._sleep, one workgroup each) captured
as a fork / join; replay time ~N means concurrent branches, ~2N serialized.
python tools/micro/graph_branches.py  (env knobs of the HIP runtime apply)."""
import os
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    cyc = int(os.environ.get("SPIN_CYCLES", "2000000"))
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    x = torch.zeros(1, device=dev)

    def step():
        s1.wait_stream(s0)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        s0.wait_stream(s1)
        x.add_(1)

    def serial():
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        x.add_(1)

    for name, fn in (("one", lambda: (torch.cuda._sleep(cyc), x.add_(1))), ("serial", serial), ("fork", step)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(50):
            g.replay()
        torch.cuda.synchronize()
        gt = (time.perf_counter() - t) / 50 * 1e6
        t = time.perf_counter()
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        et = (time.perf_counter() - t) / 50 * 1e6
        print(f"{name:7s} graph {gt:8.1f} us   eager {et:8.1f} us")


if __name__ == "__main__":
    main()
