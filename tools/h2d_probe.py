"""Decompose the PCIe-inclusive step time (bench.py pcie_inclusive): resident
batches with one graph per step, the loader's copies alone, and loader + graphs."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench


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
    out = {}
    for depth, mode in ((3, "kernel"), (3, "dma"), (3, "side"), (4, "kernel")):
        ld = ColumnarLoader(ds, B, dev, depth=depth, copy=mode)
        depth = f"{depth}_{mode}"
        nd = ld.depth
        for s, _ in ld.iter_slots():
            step(ld.slot_views(s))
        torch.cuda.synchronize()
        graphs = []
        for k in range(nd):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                step(ld.slot_views(k))
            graphs.append(gr)
        # (a) resident, one graph per step
        torch.cuda.synchronize(); t = time.perf_counter()
        for i in range(nb):
            graphs[i % nd].replay()
        torch.cuda.synchronize(); out[f"resident_graph_per_step_ms_d{depth}"] = (time.perf_counter() - t) / nb * 1e3
        # (b) copies only
        ld.prepare_epoch(); torch.cuda.synchronize(); t = time.perf_counter()
        for s, _ in ld.iter_slots():
            pass
        torch.cuda.synchronize(); out[f"copies_only_ms_d{depth}"] = (time.perf_counter() - t) / nb * 1e3
        # (c) loader + graphs, host time of the loop vs device
        ld.prepare_epoch(); torch.cuda.synchronize(); t = time.perf_counter()
        for s, _ in ld.iter_slots():
            graphs[s].replay()
        th = time.perf_counter() - t
        torch.cuda.synchronize(); out[f"loader_graph_ms_d{depth}"] = (time.perf_counter() - t) / nb * 1e3
        out[f"loader_graph_host_loop_ms_d{depth}"] = th / nb * 1e3
    # (d) raw pinned H2D of one record
    h = torch.empty(655360, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(655360, dtype=torch.uint8, device=dev)
    for _ in range(5):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(100):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); out["raw_h2d_655KB_us"] = (time.perf_counter() - t) / 100 * 1e6
    print(json.dumps({k: round(v, 4) for k, v in out.items()}))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
