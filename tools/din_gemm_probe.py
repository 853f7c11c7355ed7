"""Which mrec_gemm_multi launches does a C4 DIN train step issue (shapes, phase,
split-K)?  Eager steps (no graph); prints each launch's jobs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench
from pytorchrec_amd import dense as D
from pytorchrec_amd.loss import BCEWithLogitsLoss

orig_run = D._run


def run(jobs):
    print("gemm_multi (M, N, K, split_k, phase):",
          [(*j.args[0:3], j.args[8], j.phase) for j in jobs], flush=True)
    return orig_run(jobs)


D._run = run


class A:
    batch, lr = 4096, 0.01


dev = torch.device("cuda:0")
model, _, _, _ = bench.build_din(A, dev)
model.compile(torch.optim.SGD(model.get_parameters(), lr=A.lr), BCEWithLogitsLoss(), [], dev)
for s in range(2):
    print("step", s, flush=True)
    model.train_step(bench.din_batch(A, s, dev))
torch.cuda.synchronize()
