"""Phase clocks of the fused DIN attention backward (workgroup 0, s_memtime) in a
C4 train step: python tools/din_stamps.py (MREC_DA_STAMP_FWD=1: the wave forward's).  Prints per-sample phase durations in
clock cycles and the step's samples-per-workgroup count."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--model", "din", "--no-cpu-baseline"]
import bench  # noqa: E402
from pytorchrec_amd import _mrec  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda:0")
    model, *_ = bench.build_din(args, dev)
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    model.compile(torch.optim.SGD(model.get_parameters(), lr=args.lr), BCEWithLogitsLoss(), [], dev)
    for b in model.embedding_banks():
        b.check_ids = False
    data = bench.din_batch(args, 0, dev)
    for _ in range(3):
        model.train_step(data)
    torch.cuda.synchronize()
    buf = torch.zeros(64, dtype=torch.int64, device=dev)
    fn = _mrec.lib().mrec_din_att_debug_stamps
    fn.argtypes = [ctypes.c_void_p]
    fn(buf.data_ptr())
    model.train_step(data)
    torch.cuda.synchronize()
    fn(None)
    st = buf.cpu().tolist()
    print("stage weights:", st[1] - st[0])
    if st[60]:
        print("  zero", st[60] - st[0], " loads issued", st[61] - st[60], " W1 converted",
              st[62] - st[61], " W2 + sync", st[1] - st[62])
    if os.environ.get("MREC_DA_STAMP_FWD") == "1":  # the wave forward (wave 0's samples)
        names = ["loads+K", "row tiles", "softmax", "pool parts", "top"]
        prev = st[1]
        for k in range(7):
            base = 2 + 8 * k
            if st[base + 4] == 0:
                break
            row = [st[base] - prev] + [st[base + j] - st[base + j - 1] for j in range(1, 5)]
            prev = st[base + 4]
            print(f"sample {k}: " + "  ".join(f"{n}={v}" for n, v in zip(names, row)),
                  " total", sum(row))
        return
    if os.environ.get("MREC_DIN_BWD_ONE") == "1":  # one sample per iteration, 6 stamps
        names = ["ph0 X/g", "ph1 L1", "ph2 L2/dZ2", "ph3 dH1/dW2", "ph4 dX/dW1", "dq+next"]
    else:  # two samples per iteration, 3 stamps
        names = ["X built", "L1-L2-dH1 own rows", "dW2 dX dW1"]
    prev = st[1]
    for k in range(7):
        base = 2 + 8 * k
        if st[base + len(names) - 1] == 0:
            break
        row = []
        for j in range(len(names)):
            row.append(st[base + j] - prev)
            prev = st[base + j]
        print(f"iteration {k}: " + "  ".join(f"{n}={v}" for n, v in zip(names, row)),
              " total", sum(row))

if __name__ == "__main__":
    main()
