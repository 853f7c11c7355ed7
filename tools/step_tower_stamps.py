"""Per-workgroup phase stamps of the fused tower INSIDE a training step (bench.py's
model and batches, eager steps): ``python tools/step_tower_stamps.py [--model
deepfm|dcnv2|din]``.  Prints each stamped phase's time from the launch's first stamp
(min / median / max over the workgroups, us; 100 MHz wall clock)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorchrec_amd import _mrec  # noqa: E402
from pytorchrec_amd.loss import BCEWithLogitsLoss  # noqa: E402


def main():
    args = bench.parse()
    if args.rows_per_table is None:
        args.rows_per_table = 38462
    dev = torch.device("cuda", 0)
    build = {"deepfm": bench.build_deepfm, "dcnv2": bench.build_dcnv2, "din": bench.build_din}
    model, sparse, dense_cols, label_col = build[args.model](args, dev)
    model.compile(torch.optim.SGD(model.get_parameters(), lr=args.lr), BCEWithLogitsLoss(), [], dev)
    for bank in model.embedding_banks():
        bank.check_ids = False
    if args.model == "din":
        datas = [bench.din_batch(args, s, dev) for s in range(2)]
    else:
        bufs = [bench.make_batch_buffer(args, sparse, s, dev) for s in range(2)]
        datas = [bench.batch_views(b, args, sparse, dense_cols, label_col) for b in bufs]
    for k in range(5):
        model.train_step(datas[k % 2])
    torch.cuda.synchronize()
    grid = (args.batch + 15) // 16
    st = torch.zeros(grid, 16, dtype=torch.int64, device=dev)
    fn = _mrec.lib().mrec_tower_debug_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p], None
    fn(st.data_ptr())
    model.train_step(datas[1])
    fn(None)
    torch.cuda.synchronize()
    t = st.cpu().double() * 10.0 / 1e3
    t0 = t[:, 0].min()
    names = {0: "start", 1: "x0 loaded", 15: "cross fwd", 2: "fwd1", 3: "fwd2", 4: "fwd3",
             5: "head dot", 13: "dh_L (w0)", 14: "parts (w0)", 6: "head", 7: "bwd_L",
             8: "bwd_L-1", 9: "bwd_L-2", 10: "bwd_L-3", 11: "bwd done", 12: "ticket"}
    for k, n in names.items():
        if bool((st[:, k] != 0).all()):
            c = t[:, k] - t0
            print(f"{n:>10}: min {float(c.min()):7.2f} med {float(c.median()):7.2f} "
                  f"max {float(c.max()):7.2f} us")


if __name__ == "__main__":
    main()
