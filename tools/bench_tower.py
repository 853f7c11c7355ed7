"""Time one mrec_tower_fwd_bwd launch at a tower shape (default: C2, B=4096,
429 -> 400 -> 400 -> 400 -> 1): 100 launches captured in a HIP graph, HIP events on
the launch stream.  Prints us per launch and the weight-stream rate per CU."""
import argparse
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorchrec_amd import _mrec, dense as D  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=4096)
p.add_argument("--widths", default="429,400,400,400")
p.add_argument("--reps", type=int, default=100)
p.add_argument("--rowmajor", action="store_true", help="row-major operand outputs (kfrag off)")
p.add_argument("--cold", action="store_true", help="128 MB fill before every launch (timed with it)")
p.add_argument("--reemit", action="store_true", help="re-emit the weight images before every launch")
p.add_argument("--no-cluster", action="store_true", help="the 16-row kernel (no cluster workspace)")
args = p.parse_args()
widths = [int(x) for x in args.widths.split(",")]
B, L = args.batch, len(widths) - 1
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
Ws = [(torch.randn(widths[l + 1], widths[l], generator=g) / widths[l] ** 0.5).to(dev) for l in range(L)]
bs = [(torch.randn(widths[l + 1], generator=g) * 0.1).to(dev) for l in range(L)]
hw = (torch.randn(widths[-1], generator=g) / widths[-1] ** 0.5).to(dev)
x0 = torch.zeros(B, D._r8(widths[0]), dtype=torch.bfloat16, device=dev)
x0[:, :widths[0]] = torch.randn(B, widths[0], generator=g).to(torch.bfloat16).to(dev)
y = (torch.rand(B, generator=g) < 0.3).float().to(dev)
imgs = [D.tower_images(W) for W in Ws]
kfrag = "--rowmajor" not in sys.argv  # the training step's layout: k-fragment images
if kfrag:
    kf = lambda n: torch.empty(int(_mrec.lib().mrec_kfrag_elems(B, n)), dtype=torch.bfloat16,  # noqa: E731
                               device=dev)
    hs = [kf(widths[l + 1]) for l in range(L - 1)]
    dhs = [kf(widths[l + 1]) for l in range(L)]
    x0_img = kf(widths[0])
else:
    hs = [D._alloc(B, widths[l + 1], torch.bfloat16, dev) for l in range(L - 1)]
    dhs = [D._alloc(B, widths[l + 1], torch.bfloat16, dev) for l in range(L)]
dx0 = D._alloc(B, widths[0], torch.bfloat16, dev)
dz = torch.empty(B, device=dev)
H = widths[-1]
npart = int(_mrec.lib().mrec_ctr_head_parts(B))
part = torch.empty(npart, D._r8(H + 1), device=dev)
lp = torch.empty(npart, device=dev)
loss = torch.empty(1, device=dev)
a = _mrec.TowerArgs()
a.batch, a.n_layers = B, L
for l in range(L + 1):
    a.width[l] = widths[l]
a.x0, a.ld_x0 = x0.data_ptr(), x0.stride(0)
for l in range(L):
    a.w_fwd[l], a.w_bwd[l] = imgs[l][0].data_ptr(), imgs[l][1].data_ptr()
    a.bias[l] = bs[l].data_ptr()
    a.dh_out[l], a.ld_dh[l] = dhs[l].data_ptr(), dhs[l].stride(0)
    if l < L - 1:
        a.h_out[l], a.ld_h[l] = hs[l].data_ptr(), hs[l].stride(0)
a.head_w, a.y = hw.data_ptr(), y.data_ptr()
a.dx0, a.ld_dx0 = dx0.data_ptr(), dx0.stride(0)
a.dz, a.part, a.ldp = dz.data_ptr(), part.data_ptr(), part.stride(0)
a.loss_part, a.ticket, a.loss = lp.data_ptr(), D._ticket(dev).data_ptr(), loss.data_ptr()
if kfrag:
    a.kfrag, a.x0_img = 1, x0_img.data_ptr()
cluster = not args.no_cluster
if cluster:
    D.TOWER_CLUSTER = True
    cws = D.tower_cluster_ws(dev, B)
    a.cl_ws, a.cl_ws_bytes = cws.data_ptr(), cws.numel()


flush = torch.empty(128 << 20, dtype=torch.uint8, device=dev) if "--cold" in sys.argv else None
reemit = "--reemit" in sys.argv


def launch():
    if flush is not None:  # evict L2 and most of the Infinity Cache before each launch
        flush.fill_(1)
    if reemit:  # the step's SGD rewrites the weight images before the next tower
        for W, im in zip(Ws, imgs):
            _mrec.call("mrec_tower_weight_prep", W.data_ptr(), W.shape[0], W.shape[1], W.stride(0),
                       im[0].data_ptr(), im[1].data_ptr(), _mrec.stream_handle())
    _mrec.call("mrec_tower_fwd_bwd", ctypes.byref(a), _mrec.stream_handle())


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    launch()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(args.reps):
            launch()
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    gr.replay()
    e1.record(s)
e1.synchronize()
us = e0.elapsed_time(e1) / args.reps * 1e3
wbytes = sum(int(im[0].numel() + im[1].numel()) * 2 for im in imgs)
flops = 2 * B * sum(widths[l] * widths[l + 1] for l in range(L)) * 2
print(json.dumps({"widths": widths, "batch": B, "cluster": cluster, "us": round(us, 2),
                  "weight_stream_GBps_per_CU": round(wbytes / (us * 1e-6) / 1e9, 1),
                  "TFLOPs": round(flops / (us * 1e-6) / 1e12, 1)}))

# ---- phase stamps of one launch (diagnostic build hook) ------------------------
NS = 32 if cluster else 16
grid = ((B + 63) // 64) * 4 if cluster else (B + 15) // 16
st = torch.zeros(grid, NS, dtype=torch.int64, device=dev)
fn = _mrec.lib().mrec_tower_debug_stamps
fn.argtypes, fn.restype = [ctypes.c_void_p], None
for _ in range(3):
    launch()
fn(st.data_ptr())
launch()
fn(None)
torch.cuda.synchronize()
t = st.cpu().double() * 10.0 / 1e3  # 100 MHz ticks -> us
t0 = t[:, 0].min()
if cluster:
    names = {0: "start", 1: "x0 in"}
    for l in range(min(L, 3)):
        names.update({2 + 4 * l: f"fwd{l} poll", 3 + 4 * l: f"fwd{l} peers in",
                      4 + 4 * l: f"fwd{l} done", 5 + 4 * l: f"fwd{l} published"})
    names.update({14: "z published", 15: "z peers in", 16: "dh_L published", 31: "end"})
    for j, l in enumerate(range(L - 1, -1, -1)):
        sb = 17 + 4 * j
        names.update({sb: f"bwd{l} poll", sb + 1: f"bwd{l} peers in", sb + 2: f"bwd{l} done",
                      sb + 3: f"bwd{l} published"})
    names = {k: v for k, v in names.items() if k < 32}
    order = sorted(names)
else:
    names = {0: "start", 1: "x0 loaded", 2: "fwd1", 3: "fwd2", 4: "fwd3", 5: "head dot",
             13: "dh_L (w0)", 14: "parts (w0)", 6: "head",
             7: "bwd_L", 8: "bwd_L-1", 9: "bwd_L-2", 10: "bwd_L-3", 11: "bwd done", 12: "ticket"}
    order = (0, 1, 2, 3, 4, 5, 13, 14, 6, 7, 8, 9, 10, 11, 12)
used = [k for k in order if k in names and bool((st[:, k] != 0).all())]
rows = []
for k in used:
    col = t[:, k] - t0
    rows.append(f"{k:3d} {names.get(k, k):>18}: min {float(col.min()):7.2f} med {float(col.median()):7.2f} max {float(col.max()):7.2f} us")
print("\n".join(rows))
