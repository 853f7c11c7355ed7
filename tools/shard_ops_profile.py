"""Where the row-sharded step's runtime memsets / copies come from (VERDICT r03
item 5): a few EAGER sharded DeepFM C2 steps at world 1 with the collectives
forced (RCCL, one rank) under torch.profiler, printing every CPU op that issued a
hipMemsetAsync / hipMemcpyAsync (grouped by Python stack) and the GPU kernel
counts per step.  Usage (GPU box):

  python tools/shard_ops_profile.py [--exchange compact|slot] [--steps 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--exchange", default="compact", choices=["compact", "slot"])
    p.add_argument("--steps", type=int, default=4)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    args = bench.parse([f"--exchange={a.exchange}", "--shard", "--force-collectives"])
    from pytorchrec_amd.sharding import ShardComm
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    comm = ShardComm(force_collectives=True)
    model, sparse, dense_cols, label_col = bench.build_deepfm(args, dev, comm)
    model.compile(torch.optim.SGD(model.get_parameters(), lr=args.lr), BCEWithLogitsLoss(), [], dev)
    for b in model.embedding_banks():
        b.check_ids = False
    bufs = [bench.make_batch_buffer(args, sparse, s, dev) for s in range(2)]
    datas = [bench.batch_views(b, args, sparse, dense_cols, label_col) for b in bufs]
    for i in range(3):
        model.train_step(datas[i % 2])
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(a.steps):
            model.train_step(datas[i % 2])
        torch.cuda.synchronize()
    ev = prof.key_averages(group_by_stack_n=12)
    keys = ("Memset", "Memcpy", "memset", "memcpy", "aten::zero_", "aten::fill_", "aten::copy_",
            "aten::zeros", "aten::index", "aten::cat", "aten::stack")
    print(f"== per-step counts over {a.steps} steps (exchange {a.exchange})")
    for e in sorted(ev, key=lambda e: -e.count):
        if any(k in e.key for k in keys):
            print(f"{e.count / a.steps:6.2f}/step  {e.key}")
            for fr in (e.stack or [])[:12]:
                if "site-packages" not in fr:
                    print(f"            {fr}")
    print("== GPU kernels per step")
    agg = prof.key_averages()
    for e in sorted(agg, key=lambda e: -e.device_time_total):
        if e.device_time_total > 0 and e.count:
            print(f"{e.count / a.steps:6.2f}/step {e.device_time_total / a.steps:9.1f} us/step  {e.key[:110]}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
