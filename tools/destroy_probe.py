"""Probe: does torch.distributed.destroy_process_group() return after an RCCL
collective was captured in a HIP graph?  One variant per process (run each under
`timeout`):

    python tools/destroy_probe.py <variant>

  eager        all_reduce eagerly, destroy                       (control)
  graph_keep   capture + replay, destroy while the graph is alive
  graph_del    capture + replay, del graph + gc + sync, destroy
  graph_reset  capture + replay, graph.reset(), del, sync, destroy
  graph_abort  capture + replay, del graph, abort the communicator instead
Prints one line per phase with wall times.
"""
import gc
import os
import sys
import time

import torch
import torch.distributed as dist


def log(msg, t0=[time.perf_counter()]):
    print(f"{time.perf_counter() - t0[0]:8.3f}s {msg}", flush=True)


def main():
    v = sys.argv[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    log(f"init ({v})")
    x = torch.ones(1 << 16, device=dev)
    y = torch.empty_like(x)

    def coll():
        # all_to_all_single issues an RCCL kernel even at world 1 (the sharded
        # exchange of bench.py --force-collectives); all_reduce is a no-op there
        dist.all_to_all_single(y, x)
        dist.all_reduce(x)

    coll()
    torch.cuda.synchronize()
    log("eager all_reduce")
    g = None
    if v != "eager":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            coll()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            coll()
        g.replay()
        torch.cuda.synchronize()
        log("captured + replayed")
    if v in ("graph_del", "graph_reset", "graph_abort"):
        if v == "graph_reset":
            g.reset()
        del g
        g = None
        gc.collect()
        torch.cuda.synchronize()
        log("graph released")
    if v == "graph_abort":
        pg = dist.group.WORLD
        backend = pg._get_backend(dev)
        backend.abort() if hasattr(backend, "abort") else dist.distributed_c10d._abort_process_group()
        log("aborted")
    else:
        dist.destroy_process_group()
        log("destroyed")
    log("exit")


if __name__ == "__main__":
    main()
