"""Experiment: stage the NEXT batch inside each step's HIP graph, on a parallel
branch (forked capture stream), from a fixed pinned staging record per graph that
the host refills two steps later.  Compare with the loader's in-stream stage."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from pytorchrec_amd import _mrec


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, sparse, dense_cols, label_col = bench.build_deepfm(args, dev)
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    model.compile(torch.optim.SGD(model.get_parameters(), lr=args.lr), BCEWithLogitsLoss(), [], dev)
    model.embeddings.check_ids = False
    step = lambda d: model.train_step(d)["loss"]
    from pytorchrec_amd.loader import ColumnarDataset, ColumnarLoader
    B, nb = args.batch, 64
    g = torch.Generator().manual_seed(7)
    cols = {c.feature_name: torch.randint(0, c.category_num, (B * nb,), generator=g, dtype=torch.int32) for c in sparse}
    for c in dense_cols:
        cols[c.feature_name] = torch.rand(B * nb, generator=g)
    cols[label_col.feature_name] = (torch.rand(B * nb, generator=g) < 0.25).float()
    ds = ColumnarDataset(cols, dense_group=[c.feature_name for c in dense_cols])
    ld = ColumnarLoader(ds, B, dev, depth=2)
    for s, _ in ld.iter_slots():
        step(ld.slot_views(s))
    host = ld._host  # packed epoch (pinned)
    nbytes = ld.layout.record_bytes
    staging = torch.empty(2, nbytes, dtype=torch.uint8, pin_memory=True)
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    graphs = []
    for k in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, capture_error_mode="thread_local"):
            cs = torch.cuda.current_stream()
            side.wait_stream(cs)
            with torch.cuda.stream(side):  # branch: stage batch j+1 into the other slot
                _mrec.call("mrec_batch_stage_ex", ld._slots[1 - k].data_ptr(),
                           staging[k].data_ptr(), nbytes, ld.layout.widen_bytes, side.cuda_stream)
            step(ld.slot_views(k))
            cs.wait_stream(side)
        graphs.append(gr)
    done = [torch.cuda.Event(), torch.cuda.Event()]
    _mrec.call("mrec_batch_stage_ex", ld._slots[0].data_ptr(), host[0].data_ptr(), nbytes,
               ld.layout.widen_bytes, cur.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for j in range(nb):
        k = j % 2
        done[k].synchronize()  # graph j-2 finished reading staging[k]
        if j + 1 < nb:
            staging[k].copy_(host[j + 1])
        graphs[k].replay()
        done[k].record()
    th = time.perf_counter() - t
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    out = {"graph_branch_stage_ms": el / nb * 1e3, "host_loop_ms": th / nb * 1e3}
    # correctness spot check: slot 1 now holds the last staged batch (nb-1 odd)
    out["last_slot_ok"] = bool(torch.equal(ld._slots[(nb - 1) % 2].cpu(), host[nb - 1]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
