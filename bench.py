#!/usr/bin/env python
"""DeepFM Criteo-shaped train-step throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model deepfm|dcnv2|din]

One step = one full training step (interact fwd -> MLP fwd -> head + BCE ->
MLP bwd -> embedding sorted-segment backward, with SGD fused into every
parameter's backward kernel) over one synthetic Criteo-shaped batch (SURVEY.md
§8(d)) that is already resident in HBM.  The step is captured as a HIP graph per
pre-generated batch (4 batches, used in place) and the graphs are replayed in turn.

For N > 1 one process runs per GPU: either torch.distributed.run starts them
(WORLD_SIZE set, must equal --gpus) or ``bench.py --gpus N`` starts them itself
(``launch``: subprocess children, rank 0's line relayed).  N > 1 defaults to the C5
workload (100M-row tables); the tables are row-sharded over the ranks and the
dense tower is data-parallel (RCCL all-to-all / all-reduce inside the captured
step); each rank trains on its own 4096 samples (weak scaling) and the MAX
elapsed time over ranks is reported.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

CRITEO_FIELDS = 26
CRITEO_DENSE = 13
CRITEO_ROWS = 38462  # ceil(1,000,000 / 26), SURVEY.md §8(d) C2
C5_ROWS = 100_000_000  # rows per table, SURVEY.md §8(d) C5 (row-sharded over the ranks)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--model", default="deepfm", choices=["deepfm", "dcnv2", "din"])
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--rows-per-table", type=int, default=None,
                   help="rows of each of the 26 tables (default: 38,462 at N=1 = C2; "
                        "100,000,000 at N>1 = C5)")
    p.add_argument("--zipf", type=float, default=0.0, help="Zipf alpha for ids (0 = uniform)")
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--graph-steps", type=int, default=4,
                   help="consecutive train steps (one per resident batch) captured in one HIP "
                        "graph: one graph launch per G steps instead of per step")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--standalone-roofline", action="store_true",
                   help="also time the embedding kernels launched alone (frac_standalone)")
    p.add_argument("--no-h2d", action="store_true",
                   help="skip the PCIe-inclusive (host-fed columnar loader) measurement")
    p.add_argument("--shard", action="store_true",
                   help="row-sharded tables + DP even at N=1 (always on for N>1)")
    p.add_argument("--shard-cap", type=int, default=None,
                   help="exchange slots per (owner, table); default: sharding.default_cap "
                        "(uniform ids), min(batch, 8192 / W) with --zipf")
    p.add_argument("--force-collectives", action="store_true",
                   help="issue the all-to-alls / all-reduce even at N=1 (RCCL capture check)")
    p.add_argument("--table-dtype", default="bf16", choices=["bf16", "fp32"],
                   help="embedding tables (DeepFM / DCN-v2); the tower computes in bf16 either way")
    p.add_argument("--exchange", default="auto", choices=["auto", "compact", "slot"],
                   help="row-sharded exchange: auto = compact at N>1, slot at N=1; compact = "
                        "one record per distinct id even at N=1; slot = one row per lookup")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N > 1 collectives: nccl (= RCCL, the measured path) or gloo (a "
                        "rehearsal of the process-level protocol: eager, staged via host)")
    p.add_argument("--same-gpu", action="store_true",
                   help="rehearsal on a one-GPU box: every rank on cuda:0 (needs "
                        "--dist-backend gloo; RCCL refuses two ranks on one device)")
    p.add_argument("--stub-step", action="store_true",
                   help="launcher check without a GPU: each rank's step is one gloo all-reduce")
    args = p.parse_args(argv)
    if args.rows_per_table is None:
        # N = 1: C2 (~1M rows); N > 1: C5, 100M-row tables row-sharded over the ranks
        args.rows_per_table = C5_ROWS if args.gpus > 1 else CRITEO_ROWS
    return args


# ----------------------------------------------------------------------------
# launcher: `bench.py --gpus N` without torch.distributed.run
# ----------------------------------------------------------------------------

def launch(args) -> int:
    """One child process per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, a
    free 127.0.0.1 port), started with subprocess from this parent, which never
    touches the GPU (no exec).  Rank 0's JSON line is relayed on stdout; if any rank
    fails the others are stopped (by PID) and the parent exits non-zero."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else
                                      subprocess.DEVNULL))
    # rank 0's stdout is drained while the ranks run (a reader thread), so a child
    # that prints more than a pipe buffer never blocks on a full pipe
    import threading
    out_chunks = []
    reader = threading.Thread(target=lambda: out_chunks.extend(iter(
        lambda: procs[0].stdout.read1(65536), b"")), daemon=True)
    reader.start()
    rc = 0
    try:
        while True:
            alive = False
            for r, pr in enumerate(procs):
                code = pr.poll()
                if code is None:
                    alive = True
                elif code != 0 and rc == 0:
                    rc = code
                    print(f"bench: rank {r} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
            if not alive:
                break
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    reader.join(timeout=30)
    out0 = b"".join(out_chunks)
    lines = [ln for ln in out0.decode(errors="replace").splitlines() if ln.startswith("{")]
    if rc == 0 and lines:
        print(lines[-1], flush=True)
    elif rc == 0:
        print("bench: rank 0 printed no JSON line", file=sys.stderr, flush=True)
        rc = 1
    return rc


# ----------------------------------------------------------------------------
# workload
# ----------------------------------------------------------------------------

def _table_dtype(args):
    return torch.float32 if getattr(args, "table_dtype", "bf16") == "fp32" else torch.bfloat16


def build_deepfm(args, device, comm=None):
    """C2 DeepFM; with ``comm`` the tables are row-sharded over its ranks (each rank
    allocates only its shard) and the dense tower is data-parallel."""
    import contextlib
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DeepFM
    from pytorchrec_amd.sharding import sharded_tables
    sparse = [CategoricalColumnWithIdentity(args.rows_per_table, f"c_c_C{f + 1}")
              for f in range(CRITEO_FIELDS)]
    dense = [NumericColumn(f"c_n_I{j + 1}") for j in range(CRITEO_DENSE)]
    label = CategoricalColumnWithIdentity(2, "label")
    cap = args.shard_cap
    if cap is None and args.zipf > 0 and comm is not None:
        cap = args.batch  # skewed ids: no tight capacity (a large W * cap takes the
        # owner's large-batch path, sharding.owner_apply_large)
    ctx = (sharded_tables(comm, cap=cap, max_batch=args.batch) if comm is not None
           else contextlib.nullcontext())
    with ctx:
        model = DeepFM(sparse, dense, label, emb_size=16, layers=(400, 400, 400), dropout=0.0,
                       emb_dtype=_table_dtype(args), device=device, random_seed=2020)
    if comm is not None:
        model.distribute(comm)
        ex = getattr(args, "exchange", "auto")
        for b in model.embedding_banks():
            b.compact = {"auto": True, "compact": "always", "slot": False}[ex]
    return model, sparse, dense, label


def build_dcnv2(args, device, comm=None):
    """C3 DCN-v2: the C2 inputs (no first-order), 3 full-rank cross layers over
    x0 (26*16 + 13 = 429 wide) stacked with the deep MLP 400-400."""
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity, NumericColumn
    from pytorchrec_amd.model import DCNv2
    if comm is not None:
        raise SystemExit("bench.py: --model dcnv2 is single-GPU (config C3)")
    sparse = [CategoricalColumnWithIdentity(args.rows_per_table, f"c_c_C{f + 1}")
              for f in range(CRITEO_FIELDS)]
    dense = [NumericColumn(f"c_n_I{j + 1}") for j in range(CRITEO_DENSE)]
    label = CategoricalColumnWithIdentity(2, "label")
    model = DCNv2(sparse, dense, label, emb_size=16, cross_layers=3, layers=(400, 400),
                  emb_dtype=_table_dtype(args), device=device, random_seed=2020)
    return model, sparse, dense, label


DIN_ITEMS, DIN_CATES, DIN_L = 63001 + 1, 801 + 1, 50


def build_din(args, device, comm=None):
    """C4 DIN, Amazon-Electronics-shaped: item 63,001 (+PAD) and category 801
    (+PAD) tables, D=16, history L=50, attention MLP 80-40-1, top MLP 200-80-1."""
    from pytorchrec_amd.feature_column import CategoricalColumnWithIdentity
    from pytorchrec_amd.model import DIN
    if comm is not None:
        raise SystemExit("bench.py: --model din is single-GPU (config C4)")
    iid = CategoricalColumnWithIdentity(DIN_ITEMS, "iid")
    cid = CategoricalColumnWithIdentity(DIN_CATES, "cid")
    his = CategoricalColumnWithIdentity(DIN_ITEMS, "pos_his")
    hcat = CategoricalColumnWithIdentity(DIN_CATES, "pos_his_cate")
    label = CategoricalColumnWithIdentity(2, "label")
    model = DIN(iid, cid, his, hcat, label, emb_size=16, att_layers=(80, 40), layers=(200, 80),
                emb_dtype=torch.bfloat16, device=device, random_seed=2020)
    return model, None, None, label


def din_batch(args, seed, device):
    """Uniform ids (seeds 0..3), history lengths U{1..50}, tail-padded with 0
    (interaction_history_list.py:17-29), labels Bernoulli(0.25)."""
    B = args.batch
    g = torch.Generator().manual_seed(seed)
    iid = torch.randint(1, DIN_ITEMS, (B,), generator=g, dtype=torch.int32)
    cid = torch.randint(1, DIN_CATES, (B,), generator=g, dtype=torch.int32)
    his = torch.randint(1, DIN_ITEMS, (B, DIN_L), generator=g, dtype=torch.int32)
    hcat = torch.randint(1, DIN_CATES, (B, DIN_L), generator=g, dtype=torch.int32)
    lens = torch.randint(1, DIN_L + 1, (B, 1), generator=g)
    pad = torch.arange(DIN_L)[None, :] >= lens
    his[pad] = 0
    hcat[pad] = 0
    label = (torch.rand(B, generator=g) < 0.25).float()
    return {"iid": iid.to(device), "cid": cid.to(device), "pos_his": his.to(device),
            "pos_his_cate": hcat.to(device), "pos_his_len": lens.reshape(-1).to(device),
            "label": label.to(device)}


def zipf_ids(rng, alpha, n, size):
    """Truncated Zipf ids in [0, n): P(id = k - 1) proportional to k^-alpha, k = 1..n
    (SURVEY.md §8(d)'s Zipf variant).  Exact inverse CDF up to 2^22 rows, the
    continuous approximation above (C5's 100M-row tables).  Clipping an unbounded
    numpy zipf draw to n - 1 instead would pile the tail's mass (~57 % of the
    lookups at alpha 1.05, n = 38462) onto the last row."""
    import numpy as np
    u = rng.random(size)
    if n <= (1 << 22):
        cdf = np.cumsum(np.arange(1, n + 1, dtype=np.float64) ** -alpha)
        return np.minimum(np.searchsorted(cdf / cdf[-1], u, side="right"), n - 1)
    e = 1.0 - alpha
    k = np.floor((1.0 + u * ((n + 1.0) ** e - 1.0)) ** (1.0 / e)) - 1.0
    return np.clip(k, 0, n - 1).astype(np.int64)


def make_batch_buffer(args, sparse, seed, device):
    """One contiguous byte buffer per batch: ids [F, B] int32 | dense [B, 13] f32 |
    label [B] f32; returns (buffer, views-builder)."""
    B, F = args.batch, len(sparse)
    g = torch.Generator(device="cpu").manual_seed(seed)
    if args.zipf > 0:
        import numpy as np
        rng = np.random.default_rng(seed + 1)
        ids = torch.from_numpy(np.stack([zipf_ids(rng, args.zipf, c.category_num, B)
                                         for c in sparse]).astype("int32"))
    else:
        ids = torch.stack([torch.randint(0, c.category_num, (B,), generator=g, dtype=torch.int32)
                           for c in sparse])
    dense = torch.rand(B, CRITEO_DENSE, generator=torch.Generator().manual_seed(seed + 2))
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed + 3)) < 0.25).float()
    parts = [ids.reshape(-1).view(torch.uint8), dense.reshape(-1).view(torch.uint8),
             label.view(torch.uint8)]
    return torch.cat(parts).to(device)


def batch_views(buf, args, sparse, dense_cols, label_col):
    B, F = args.batch, len(sparse)
    n_ids = F * B * 4
    n_dense = B * CRITEO_DENSE * 4
    ids = buf[:n_ids].view(torch.int32).view(F, B)
    dense = buf[n_ids:n_ids + n_dense].view(torch.float32).view(B, CRITEO_DENSE)
    label = buf[n_ids + n_dense:n_ids + n_dense + B * 4].view(torch.float32)
    data = {c.feature_name: ids[f] for f, c in enumerate(sparse)}
    data["__dense__"] = dense
    data[label_col.feature_name] = label
    return data


# ----------------------------------------------------------------------------
# per-kernel roofline (HIP events on the launch stream, eager back-to-back launches)
# ----------------------------------------------------------------------------

def time_launches(fn, reps=100):
    """Average device time of one launch of ``fn``: ``reps`` back-to-back launches
    captured in a HIP graph (no host launch overhead), bracketed by HIP events on
    the stream the kernels run on."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        # thread_local: the RCCL watchdog thread queries its events during the capture
        # (a sharded model's process group); "global" mode made that query fail and abort
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(reps):
                fn()
        g.replay()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
    e1.synchronize()
    torch.cuda.current_stream().wait_stream(s)
    return e0.elapsed_time(e1) / reps * 1e-3  # seconds per launch


def instep_kernel_times(step, datas, names, steps=4, replays=30, strip_coreduce=False,
                        comm=None):
    """Device time of every launch of the named libmrec entry points INSIDE the
    graph-replayed training step: ``steps`` train steps (batch i % len(datas)) are
    captured in one HIP graph with the kernel clock on (mrec_kernel_clock: clocked
    instantiations of the hot kernels whose waves record their start and end,
    s_memrealtime at 100 MHz, into the slot each launch took at capture); the graph
    is replayed ``replays`` times.  (HIP event-record nodes spliced into the graph
    were tried first: each added 12-14 us to a 10-15 us kernel.)

    A launch's in-step time is its first wave's start to the NEXT clocked launch's
    first wave's start: the graph runs the step's kernels back to back, so this is
    the launch's share of the step -- dispatch, its waves, and the end-of-kernel
    cache write-back before the next kernel's waves can start -- which is what
    rocprof's per-kernel duration inside the replayed graph shows (its kernels
    abut).  The last launch of the graph has no successor and gives no sample.
    ``span`` is the waves' own first start to last end (the part the kernel's code
    controls); a launch whose next libmrec call is not a clocked launch (work the
    clock does not see follows it) reports its span as its in-step time.
    ``strip_coreduce``: the deferred MLP weight-gradient reductions do
    not ride in the embedding apply (they run as their own launch at the end of
    the backward) -- the apply's CoReduce share is the difference.  ``comm``: the
    row-sharded step's communicator -- its collectives (RCCL all-to-all /
    all-reduce) count as calls, so a launch followed by one reports its own waves'
    span and the collective's time stays out of every launch's share.

    Returns ({name: median in-step seconds}, {name: median span seconds},
    median seconds from the first clocked start to the last clocked end / steps)."""
    import numpy as np
    from pytorchrec_amd import _mrec, dense as D
    lib = _mrec.lib()
    dev = torch.device("cuda", torch.cuda.current_device())
    n_slots = 64
    buf = torch.empty(n_slots, 4096, 16, dtype=torch.int64, device=dev)  # mrec.h MREC_KCLOCK_*
    tags, at_call = [], []  # per clock slot: entry point, index of the libmrec call
    calls = [0]
    real_call, real_take = _mrec.call, D.take_pending
    capturing = [False]

    def spy(name, *a):
        if not capturing[0]:
            return real_call(name, *a)
        before = int(lib.mrec_kernel_clock_used())
        r = real_call(name, *a)
        k = int(lib.mrec_kernel_clock_used()) - before
        tags.extend([name] * k)
        at_call.extend([calls[0]] * k)
        calls[0] += 1
        return r

    _mrec.call = spy
    wrapped = []
    if comm is not None:
        for meth in ("exchange", "allreduce_sum_", "allreduce_mean_"):
            orig = getattr(comm, meth, None)
            if orig is None:
                continue

            def counted(*a, _o=orig, **k):
                r = _o(*a, **k)
                if capturing[0]:
                    calls[0] += 1
                return r
            setattr(comm, meth, counted)
            wrapped.append(meth)
    if strip_coreduce:
        D.take_pending = lambda n=0: []
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(2):
                step(datas[i % len(datas)])
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        lib.mrec_kernel_clock(buf.data_ptr(), n_slots)
        capturing[0] = True
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for i in range(steps):
                    step(datas[i % len(datas)])
        finally:
            capturing[0] = False
            lib.mrec_kernel_clock(None, 0)
    finally:
        _mrec.call, D.take_pending = real_call, real_take
        for meth in wrapped:
            delattr(comm, meth)  # (the instance attribute shadowed the method)
    share = {n: [] for n in names}
    span = {n: [] for n in names}
    unclocked = set()
    whole = []
    n = len(tags)
    for _ in range(replays):
        buf[..., 0].fill_(-1)  # starts: all ones (u64 max)
        buf[..., 1].zero_()
        g.replay()
        torch.cuda.synchronize()
        u = buf[:n, :, :2].cpu().numpy().view(np.uint64)
        t0, t1 = u[:, :, 0].min(axis=1), u[:, :, 1].max(axis=1)
        if n == 0 or not (t1 > t0).all():
            continue
        whole.append(float(t1[-1] - t0[0]) * 1e-8 / steps)
        for i, tag in enumerate(tags):
            if CAT_SPANS is not None and tag == EMB_PAIR[1]:  # (diagnostic build, MREC_KC_CAT)
                for c in range(4):
                    st_, en_ = u[i, c * 1024:(c + 1) * 1024, 0], u[i, c * 1024:(c + 1) * 1024, 1]
                    cs, ce = st_.min(), en_.max()
                    if ce > cs:
                        ok = en_ > 0
                        # per-wave shards (waves of one kind < 1024): start / duration
                        # quantiles over the kind's waves
                        ws_ = (st_[ok] - t0[i]).astype(np.float64) * 1e-8
                        wd_ = (en_[ok] - st_[ok]).astype(np.float64) * 1e-8
                        q = [float(x) for x in np.quantile(ws_, [0.5, 0.9, 1.0])] + \
                            [float(x) for x in np.quantile(wd_, [0.5, 0.9, 1.0])]
                        CAT_SPANS.setdefault(c, []).append(
                            (float(cs - t0[i]) * 1e-8, float(ce - t0[i]) * 1e-8, q))
            if tag in share:
                span[tag].append(float(t1[i] - t0[i]) * 1e-8)  # 100 MHz ticks
                # the share needs the next clocked launch to be the next libmrec call
                # (DCN-v2's cross layers run between its interaction and tower)
                if i + 1 < n and at_call[i + 1] == at_call[i] + 1:
                    share[tag].append(float(t0[i + 1] - t0[i]) * 1e-8)
                elif i + 1 < n:
                    unclocked.add(tag)
    g.reset()

    def med(d):
        return {k: sorted(v)[len(v) // 2] for k, v in d.items() if v}
    ms, mp = med(share), med(span)
    for k in unclocked:  # a launch followed by unclocked work: its own waves only
        ms[k] = mp[k]
    return ms, mp, (sorted(whole)[len(whole) // 2] if whole else None)


EMB_PAIR = ("mrec_interact_fwd_ex", "mrec_emb_bwd_apply_ex")
# MREC_BENCH_KC_CAT=1 with a library built with -DMREC_KC_CAT: the apply's block kinds
# (co-reduce, segment, hot-segment, single-lookup blocks) clocked apart
CAT_SPANS = {} if os.environ.get("MREC_BENCH_KC_CAT") == "1" else None
TOWER_PAIR = ("mrec_tower_fwd_bwd", "mrec_tower_dw_ex")
DIN_PAIR = ("mrec_din_att_fwd", "mrec_din_att_bwd")


def embedding_roofline(model, step, datas, args, in_step=True):
    """The bench line's ``roofline`` (HBM-bound embedding path) and
    ``roofline_kernels``.  ``achieved`` = SURVEY.md §8(d) algorithmic bytes of the
    step's two embedding launches (interaction + plan; apply) / their durations
    INSIDE the graph-replayed training step (instep_kernel_times: what rocprof's
    in-step kernel table shows, the apply including the MLP's deferred split-K
    reductions that ride in it -- their share is reported as
    ``apply_coreduce_us``, measured as the apply with them moved out).  With
    --standalone-roofline the kernels launched alone back to back are reported
    too (``frac_standalone``).  The dense tower's launches (MFMA) are timed in the
    same captured steps."""
    D = model.embeddings.dim
    first_order = bool(model.embeddings.has_w)
    es = model.embeddings.weight.element_size()
    F = model.embeddings.n_tables
    alg_fwd, alg_bwd = alg_bytes_per_sample(F, D, CRITEO_DENSE, first_order, es)
    nbytes = (alg_fwd + alg_bwd) * args.batch
    out = {}
    rk = {}
    if in_step:
        t, t_span, clocked_step = instep_kernel_times(step, datas, EMB_PAIR + TOWER_PAIR)
        # the stripped step runs the reductions as a launch of their own right after the
        # apply, so the apply's share there is not comparable: the co-reduce's cost is
        # the difference of the apply's wave spans with and without it
        span_strip = instep_kernel_times(step, datas, EMB_PAIR[1:], strip_coreduce=True)[1]
        t_strip = {EMB_PAIR[1]: t[EMB_PAIR[1]] - (t_span[EMB_PAIR[1]] - span_strip[EMB_PAIR[1]])}
        t_pair = t[EMB_PAIR[0]] + t[EMB_PAIR[1]]
        ach = nbytes / t_pair / 1e9
        t_emb = t[EMB_PAIR[0]] + t_strip[EMB_PAIR[1]]
        traffic, tsrc = pmc_traffic([EMB_PAIR[0], "mrec_emb_bwd_apply"], args)
        out["roofline"] = {
            "bound": "hbm", "kernel": "embedding path: " + " + ".join(EMB_PAIR),
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "avg_us": round(t_pair * 1e6, 3), "bytes_per_launch": nbytes,
            "bytes_rule": "SURVEY.md §8(d) algorithmic bytes per sample x batch",
            "timing": "in-step: the kernels' own clock (mrec_kernel_clock, s_memrealtime) "
                      "inside the graph-replayed train steps, each launch's first wave start "
                      "to the next launch's (its share of the step, as rocprof's abutting "
                      "in-graph durations count it); median over 4 steps x 30 replays",
            "clocked_step_us": round(clocked_step * 1e6, 3) if clocked_step else None,
            "apply_coreduce_us": round((t[EMB_PAIR[1]] - t_strip[EMB_PAIR[1]]) * 1e6, 3),
            "frac_embedding_only": round(nbytes / t_emb / 1e9 / HBM_PEAK_GBS, 4),
            "traffic_source": tsrc}
        for k in EMB_PAIR:
            rk[k] = {"avg_us": round(t[k] * 1e6, 3), "timing": "in-step",
                     "wave_span_us": round(t_span[k] * 1e6, 3)}
        rk[EMB_PAIR[1]]["avg_us_without_coreduce"] = round(t_strip[EMB_PAIR[1]] * 1e6, 3)
        if CAT_SPANS:
            rk[EMB_PAIR[1]]["block_kinds_us"] = {
                ("co_reduce", "segments", "hot", "singles")[c]: {
                    "span": [round(sorted(x[0] for x in v)[len(v) // 2] * 1e6, 2),
                             round(sorted(x[1] for x in v)[len(v) // 2] * 1e6, 2)],
                    "wave_start_p50_p90_max": [round(v[len(v) // 2][2][j] * 1e6, 2)
                                               for j in range(3)],
                    "wave_dur_p50_p90_max": [round(v[len(v) // 2][2][j] * 1e6, 2)
                                             for j in range(3, 6)]}
                for c, v in sorted(CAT_SPANS.items())}
        if args.model in ("deepfm", "dcnv2"):
            lins = [m for m in model.mlp.modules() if isinstance(m, torch.nn.Linear)]
            # DCN-v2: the cross layers (d x d) run in the same tower / tower_dw launches
            cross = list(getattr(model, "cross", []))
            widths = [lins[0].in_features] + [m.out_features for m in lins]
            dims = [(c.out_features, c.in_features) for c in cross] + \
                [(widths[l + 1], widths[l]) for l in range(len(widths) - 1)]
            mm = sum(n * k for n, k in dims)
            mm_c = sum(c.out_features * c.in_features for c in cross)
            for name, fl in ((TOWER_PAIR[0], 2 * 2 * args.batch * mm),
                             (TOWER_PAIR[1], 2 * args.batch * sum(n * (k + 1) for n, k in dims))):
                if name in t:
                    d = {"avg_us": round(t[name] * 1e6, 3), "flop": fl,
                         "TFLOP/s": round(fl / t[name] / 1e12, 1),
                         "frac_of_mfma_peak": round(fl / t[name] / 1e12 / MFMA_PEAK_TFLOPS, 4),
                         "timing": "in-step", "wave_span_us": round(t_span[name] * 1e6, 3)}
                    if name == TOWER_PAIR[0]:
                        wimg = 2 * 2 * mm  # bf16 forward + transposed images
                        d["weight_bytes_per_workgroup"] = wimg
                        d["per_CU_L2_GB/s"] = round(wimg / t[name] / 1e9, 1)
                        d["bound"] = ("per-CU L2 read rate (~70 GB/s per CU, MI355X_MICROARCH.md "
                                      "indexed-rows table)")
                        if cross:
                            ph = tower_cross_phases(step, datas[0], args.batch, len(lins))
                            if ph:
                                frac = (ph["cross_fwd_us"] + ph["cross_bwd_us"]) / ph["wave_us"]
                                tc = t[name] * frac
                                fc = 2 * 2 * args.batch * mm_c
                                d["cross"] = {
                                    "layers": len(cross), "flop": fc,
                                    "in_step_us": round(tc * 1e6, 3),
                                    "TFLOP/s": round(fc / tc / 1e12, 1),
                                    "frac_of_mfma_peak": round(fc / tc / 1e12 / MFMA_PEAK_TFLOPS, 4),
                                    "timing": "the tower's in-step time x the cross phases' share "
                                              "of the workgroups' wall clock (phase stamps of an "
                                              "eager step, medians over workgroups)",
                                    "phases_us": ph}
                                dw = 2 * args.batch * sum(n * (k + 1) for n, k in dims[:len(cross)])
                                rk.setdefault("cross_dw_share_of_tower_dw_flop", round(
                                    dw / (2 * args.batch * sum(n * (k + 1) for n, k in dims)), 4))
                    rk[name] = d
    if args.standalone_roofline or not in_step:
        ks = kernel_rooflines(model, datas[0], args)
        ts = sum(v[0] for v in ks.values())
        impl = sum(v[2] for v in ks.values())
        if "roofline" not in out:
            ach = nbytes / ts / 1e9
            traffic, tsrc = pmc_traffic(list(ks), args)
            out["roofline"] = {"bound": "hbm", "kernel": "embedding path: " + " + ".join(ks),
                               "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                               "avg_us": round(ts * 1e6, 3), "bytes_per_launch": nbytes,
                               "bytes_rule": "SURVEY.md §8(d) algorithmic bytes per sample x batch",
                               "timing": "standalone: each kernel launched alone back to back",
                               "traffic_source": tsrc}
        out["roofline"]["frac_standalone"] = round(nbytes / ts / 1e9 / HBM_PEAK_GBS, 4)
        out["roofline"]["as_implemented_bytes_per_launch"] = impl
        for k, v in ks.items():
            rk.setdefault(k, {})["standalone_avg_us"] = round(v[0] * 1e6, 3)
            rk[k]["as_implemented_bytes"] = v[2]
    att = attainable()
    if att:
        out["roofline"]["attainable"] = att
        out["roofline"]["frac_of_attainable"] = round(out["roofline"]["achieved"] / att["GB/s"], 4)
    out["roofline_kernels"] = rk
    return out


SHARD_EMB = ("mrec_shard_bucketize_dedup_ex", "mrec_shard_bucketize_dedup_q", "mrec_shard_gather_wire_ex",
             "mrec_shard_wire_unpack_ex", "mrec_interact_fwd_ex", "mrec_interact_fwd_rec",
             "mrec_emb_bwd_apply_rec", "mrec_emb_bwd_apply_wire", "mrec_emb_bwd_apply_wire_sgd")


def sharded_roofline(model, step, datas, args):
    """The row-sharded (compact exchange) line's ``roofline``, IN-STEP: the same
    SURVEY.md §8(d) algorithmic bytes as the unsharded step (the exchange adds no
    algorithmic bytes: it only moves the same rows between ranks) over the summed
    in-step time of every embedding-path launch of the step -- the sender's
    bucketize / dedup, the owner's record gather (+ its backward plan), the sender's
    unpack, the interaction (+ the sender's plan), the sender's gradient sums into
    records and the owner's apply -- each timed by its clocked instantiation inside
    the graph-replayed step (mrec_kernel_clock); the RCCL collectives are counted as
    calls, so no launch's share includes one.  The collectives' own time is the
    step's remainder (``collectives_us``)."""
    D = model.embeddings.dim
    first_order = bool(model.embeddings.has_w)
    es = model.embeddings.weight.element_size()
    F = model.embeddings.n_tables
    alg_fwd, alg_bwd = alg_bytes_per_sample(F, D, CRITEO_DENSE, first_order, es)
    nbytes = (alg_fwd + alg_bwd) * args.batch
    names = SHARD_EMB + TOWER_PAIR + ("mrec_sgd_multi",)
    t, t_span, clocked_step = instep_kernel_times(step, datas, names, comm=model.embeddings.comm)
    emb = [k for k in SHARD_EMB if k in t]
    t_emb = sum(t[k] for k in emb)
    ach = nbytes / t_emb / 1e9
    traffic, tsrc = pmc_traffic(sorted({KERNEL_OF[k] for k in emb if k in KERNEL_OF}), args)
    out = {"roofline": {
        "bound": "hbm", "kernel": "row-sharded embedding path: " + " + ".join(emb),
        "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
        "avg_us": round(t_emb * 1e6, 3), "bytes_per_launch": nbytes,
        "bytes_rule": "SURVEY.md §8(d) algorithmic bytes per sample x batch (the exchange "
                      "adds none)",
        "timing": "in-step: the kernels' own clock inside the graph-replayed train steps "
                  "(each launch's first wave start to the next libmrec launch's; a launch "
                  "followed by a collective: its own waves' span); median over 4 steps x 30 "
                  "replays",
        "clocked_step_us": round(clocked_step * 1e6, 3) if clocked_step else None}}
    if clocked_step:
        out["roofline"]["collectives_us"] = round((clocked_step - sum(t.values())) * 1e6, 3)
    out["roofline_kernels"] = {k: {"avg_us": round(t[k] * 1e6, 3), "timing": "in-step",
                                   "wave_span_us": round(t_span[k] * 1e6, 3)} for k in t}
    return out


# bench entry point -> the PMC stamp's kernel key (tools/pmc_traffic.py KERNELS)
KERNEL_OF = {"mrec_shard_bucketize_dedup_ex": "mrec_shard_bucketize_dedup",
             "mrec_shard_bucketize_dedup_q": "mrec_shard_bucketize_dedup",
             "mrec_shard_gather_wire_ex": "mrec_shard_gather_wire",
             "mrec_shard_wire_unpack_ex": "mrec_shard_wire_move",
             "mrec_interact_fwd_ex": "mrec_interact_fwd_ex",
             "mrec_interact_fwd_rec": "mrec_interact_fwd_ex",
             "mrec_emb_bwd_apply_rec": "mrec_emb_bwd_apply",
             "mrec_emb_bwd_apply_wire": "mrec_emb_bwd_apply",
             "mrec_emb_bwd_apply_wire_sgd": "mrec_emb_bwd_apply"}


def tower_cross_phases(step, data, B, L):
    """Per-workgroup phase stamps of the fused tower (mrec_tower_debug_stamps, 100
    MHz wall clock) over one eager train step: the cross network's forward (stamp 1
    -> 15) and backward (the MLP's last backward layer -> stamp 11) against the
    workgroup's whole span (0 -> 12), medians over the workgroups, in us."""
    from pytorchrec_amd import _mrec
    import ctypes
    dev = torch.device("cuda", torch.cuda.current_device())
    grid = (B + 15) // 16
    st = torch.zeros(grid, 16, dtype=torch.int64, device=dev)
    fn = _mrec.lib().mrec_tower_debug_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p], None
    torch.cuda.synchronize()
    fn(st.data_ptr())
    try:
        step(data)
    finally:
        fn(None)
    torch.cuda.synchronize()
    t = st.cpu().double() * 1e-2  # us
    last_mlp = 7 + (L - 1)  # stamp 7 + (L - 1 - l) at the MLP's first layer (l = 0)
    if not bool((st[:, [0, 1, 15, last_mlp, 11, 12]] != 0).all()):
        return None
    med = lambda x: round(float(x.median()), 3)  # noqa: E731
    return {"cross_fwd_us": med(t[:, 15] - t[:, 1]), "cross_bwd_us": med(t[:, 11] - t[:, last_mlp]),
            "wave_us": med(t[:, 12] - t[:, 0])}


def alg_bytes_per_sample(F, D, n_dense, first_order, es=2):
    """SURVEY.md §8(d) algorithmic bytes per sample, bf16 weights (es = 2; fp32
    tables es = 4), int32 ids:
    fwd = ids F*4 + useful row bytes F*(D+w)*es + dense n_dense*4 + label 4;
    bwd = ids F*4 + row-sparse read-modify-write 2*F*(D+w)*es.
    C2 DeepFM: 1,044 + 1,872 = 2,916; C3 DCN-v2 (no w): 992 + 1,768 = 2,760."""
    row = (D + (1 if first_order else 0)) * es
    return F * 4 + F * row + n_dense * 4 + 4, F * 4 + 2 * F * row


def kernel_rooflines(model, data, args):
    """Average duration of each HBM-bound embedding kernel, launched exactly as the
    train step launches it, with its algorithmic bytes (what
    ``roofline.achieved`` uses) and its as-implemented bytes.
    Measured on an unsharded bank of the model's shapes (at N>1 the model's tables
    are shards).  Returns {kernel: (seconds, algorithmic bytes, as-implemented bytes)}."""
    from pytorchrec_amd import _mrec, embedding as E
    dev = torch.device("cuda", torch.cuda.current_device())
    first_order = bool(model.embeddings.has_w)
    if type(model.embeddings) is E.EmbeddingBank:
        bank = model.embeddings  # unsharded: time the model's own bank (no second copy of
        # a 100M-row C5 bank); the timed updates run after the timed region
    else:
        # sharded model: a bank of one shard's rows (the per-GPU footprint; a second
        # full C5 bank would not fit beside the shard)
        world = max(1, int(os.environ.get("WORLD_SIZE", "1")))
        bank = E.EmbeddingBank([max(1, args.rows_per_table // world)] * CRITEO_FIELDS, 16,
                               with_first_order=first_order, dtype=_table_dtype(args), device=dev)
        E.init_bank_(bank, generator=torch.Generator(device=dev).manual_seed(5))
        bank.use_fused_sgd(args.lr)
        bank.check_ids = False
    fm = first_order  # DeepFM: FM2 + first order; DCN-v2: plain gather into x0
    dense_weight = torch.randn(CRITEO_DENSE, device=dev) * 0.01 if fm else None
    global_bias = torch.zeros(1, device=dev) if fm else None
    B, F, D = args.batch, bank.n_tables, bank.dim
    ids = model._ids(data)
    dense = model._dense(data)
    es = bank.weight.element_size()
    alg_fwd, alg_bwd = alg_bytes_per_sample(F, D, CRITEO_DENSE, first_order, es)
    w = 1 if first_order else 0
    out = {}
    with torch.no_grad():
        # the step's forward launch: interaction + the backward's hash plan in one
        # kernel (mrec_interact_fwd_ex)
        def fwd():
            E._InteractFn.forward(_Ctx(), bank.weight, dense_weight, global_bias, None,
                                  bank, ids, dense, fm, fm, model.x0_cols, torch.bfloat16,
                                  True)
        # as implemented, bytes/sample: ids F*4 + useful row bytes F*(D+w)*2 + dense
        # 13*4 + x0 write x0_cols*2 + logit 4 + fm_sum D*4; plan: ids F*4 again + per
        # lookup one 12-B workspace entry (row table / descriptor / permutation)
        impl_fwd = (F * 4 + F * (D + w) * es + CRITEO_DENSE * 4 + model.x0_cols * 2 + 4
                    + (D * 4 if fm else 0) + F * 4 + F * 12)
        t = time_launches(fwd)
        out["mrec_interact_fwd_ex"] = (t, alg_fwd * B, impl_fwd * B)

        ws, wsb = E._plan(bank, ids, 0, B, None)
        torch.cuda.synchronize()

        x0, logit = E._InteractFn.forward(_Ctx(), bank.weight, dense_weight, global_bias, None,
                                          bank, ids, dense, fm, fm, model.x0_cols,
                                          torch.bfloat16, False)
        fm_sum = torch.zeros(B, D, device=x0.device) if fm else None
        dx0 = torch.zeros_like(x0)
        dl = torch.zeros(B, device=x0.device) if fm else None

        def apply():
            E._apply(bank, ws, wsb, B, dx=dx0, dfm=dl, fm_sum=fm_sum, x0=x0 if fm else None, dw=dl)
        t = time_launches(apply)
        # as implemented, per lookup: perm/row table 4 + dx D*2 (+ v re-read D*2 for
        # the FM term) + row read+write 2*(D+w)*2; per sample: fm_sum D*4 + dlogit 4
        impl_bwd = (F * (4 + D * 2 + (D * 2 if fm else 0) + 2 * (D + w) * es)
                    + ((D * 4 + 4) if fm else 0))
        out["mrec_emb_bwd_apply"] = (t, alg_bwd * B, impl_bwd * B)
    return out


def din_rooflines(model, data, args):
    """The fused DIN attention-unit kernels (mrec_din_att_fwd / _bwd, din_att.hip),
    each launched as the train step launches it on the step's own gathered rows,
    timed with HIP events over back-to-back graph replays.  Algorithmic FLOP per
    sample (SURVEY.md §8(d) style, history positions L = 50, unit 4E=128 -> 80 -> 40
    -> 1): forward F = 2 L (128*80 + 80*40 + 40); the backward launch recomputes the
    forward and back-propagates (dX and dW: 2F) = 3F.  HBM bytes per sample: fwd
    reads q + L k rows (E=32 bf16) + L history ids, writes a (L fp32) + top (2E
    bf16); bwd reads the rows, a, dtop and writes the rows' gradient.
    Returns {kernel: (seconds, flop per launch, bytes per launch)}."""
    from pytorchrec_amd import _mrec, dense as D
    lins = D._din_att_linears(model.att_mlp, model.att_out)
    B, L, E = args.batch, DIN_L, 2 * model.emb_size
    assert D.din_att_supported(E, model.att_mlp, model.att_out)
    dev = model.embeddings.weight.device
    from pytorchrec_amd.embedding import gather
    iid = model.iid_column.get_feature_ids(data)
    cid = model.cid_column.get_feature_ids(data)
    his = model.his_column.get_feature_ids(data)
    hcat = model.his_cate_column.get_feature_ids(data)
    with torch.no_grad():
        rows = D._bf16_rows(gather(model.embeddings,
                                   [torch.cat([iid.reshape(-1), his.reshape(-1).to(iid.dtype)]),
                                    torch.cat([cid.reshape(-1),
                                               hcat.reshape(-1).to(cid.dtype)])],
                                   out_dtype=torch.bfloat16))
    his32 = his.to(torch.int32).contiguous()
    w1, w2, w3 = (D._weight_f32(m.weight) for m in lins)
    b1, b2, b3 = (m.bias.detach().float().contiguous() for m in lins)
    w3 = w3.reshape(-1)
    H1, H2 = w1.shape[0], w2.shape[0]
    a = torch.empty(B, L, dtype=torch.float32, device=dev)
    top = D._alloc(B, 2 * E, torch.bfloat16, dev)
    dtop = torch.randn(B, 2 * E, device=dev).to(torch.bfloat16)
    d_rows = D._alloc(rows.shape[0], E, torch.bfloat16, dev)
    lib = _mrec.lib()
    parts = int(lib.mrec_din_att_parts(B))
    part = torch.empty(parts, int(lib.mrec_din_att_param_count(E, H1, H2)),
                       dtype=torch.float32, device=dev)
    wargs = (w1.data_ptr(), w1.stride(0), b1.data_ptr(), H1, w2.data_ptr(), w2.stride(0),
             b2.data_ptr(), H2, w3.data_ptr(), b3.data_ptr())

    def fwd():
        _mrec.call("mrec_din_att_fwd", rows.data_ptr(), rows.stride(0), his32.data_ptr(),
                   his32.stride(0), B, L, E, *wargs, a.data_ptr(), top.data_ptr(),
                   top.stride(0), _mrec.stream_handle())

    def bwd():
        _mrec.call("mrec_din_att_bwd", rows.data_ptr(), rows.stride(0), B, L, E, *wargs,
                   a.data_ptr(), dtop.data_ptr(), dtop.stride(0), d_rows.data_ptr(),
                   d_rows.stride(0), part.data_ptr(), parts, _mrec.stream_handle())
    F = 2 * L * (4 * E * H1 + H1 * H2 + H2)
    row_b = (1 + L) * E * 2
    out = {"mrec_din_att_fwd": (time_launches(fwd, 20), F * B,
                                (row_b + L * 4 + L * 4 + 2 * E * 2) * B),
           "mrec_din_att_bwd": (time_launches(bwd, 20), 3 * F * B,
                                (2 * row_b + L * 4 + 2 * E * 2) * B)}
    return out


PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
PMC_FILE = os.path.join(PROFILES, "pmc_traffic.json")
CEIL_FILE = os.path.join(PROFILES, "ceilings.json")


def pmc_workload(args):
    """The workload key a PMC stamp must match (tools/pmc_traffic.py writes the same)."""
    return {"model": args.model, "batch": args.batch, "rows_per_table": args.rows_per_table,
            "zipf": float(args.zipf or 0.0), "shard": bool(args.shard or args.gpus > 1),
            "exchange": args.exchange if (args.shard or args.gpus > 1) else None}


def lib_digest():
    """The source digest libmrec.so was built from (pytorchrec_amd/build.py stamp)."""
    try:
        with open(os.path.join(ROOT, "pytorchrec_amd", "lib", "libmrec.so.sha256")) as fh:
            return fh.read().strip()
    except OSError:
        return None


def pmc_traffic(kernels, args):
    """HBM bytes per launch summed over ``kernels`` from the committed PMC passes
    (tools/gpu_pmc.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs of
    this bench, corrected by the calibration tools/pmc_traffic.py applies).  rocprof
    cannot count the run it is printed by, so a stamp names its profiled run: the
    traffic is reported only when that run had THIS workload (model, batch, rows per
    table, Zipf alpha, sharding / exchange) AND this library (the source digest of
    libmrec.so, i.e. the same kernels); otherwise ``traffic`` is null and the source
    says why.  Returns (bytes | None, source)."""
    src = {"file": "profiles/pmc_traffic.json"}
    try:
        with open(PMC_FILE) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None, dict(src, missing=True)
    want, lib = pmc_workload(args), lib_digest()
    runs = [r for r in pmc.get("runs", []) if r.get("workload") == want]
    if not runs:
        return None, dict(src, no_run_for=want)
    run = runs[-1]
    if run.get("lib") != lib:
        return None, dict(src, stale={"stamped_lib": run.get("lib"), "this_lib": lib,
                                      "stamped_commit": run.get("commit")})
    try:
        per = run["kernels"]
        nbytes = int(sum(per[k]["hbm_bytes_per_launch"] for k in kernels))
    except (KeyError, TypeError):
        return None, dict(src, missing_kernels=[k for k in kernels if k not in run.get("kernels", {})])
    return nbytes, dict(src, run={k: run[k] for k in ("workload", "commit", "lib", "utc")},
                        kernels={k: per[k] for k in kernels}, correction=pmc.get("correction"))


def attainable():
    """The measured ceiling the embedding path is compared with beside the spec peak:
    random 64-B row gathers from the C2-sized (64 MB, Infinity-Cache resident) table,
    bandwidth form, from the committed step-0 microbenchmark (tools/micro/ceilings.hip,
    profiles/ceilings.json)."""
    try:
        with open(CEIL_FILE) as fh:
            c = json.load(fh)
        g = [x for x in c["gather"] if x["row_bytes"] == 64 and x["table_bytes"] == 64 << 20][0]
        return {"GB/s": g["row_GB/s"], "what": "random 64-B row gather, 64 MB table, 16 M lookups",
                "stream_copy_GB/s": c["stream_copy"]["GB/s"], "file": "profiles/ceilings.json"}
    except (OSError, KeyError, ValueError, IndexError):
        return None


MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 (MI355X_MICROARCH.md)


def end_to_end(args, per_gpu_samples_s):
    """End-to-end samples/s per GPU against min(HBM, MFMA) samples/s roofline,
    SURVEY.md §8(d): HBM = 8 TB/s / algorithmic train-step bytes per sample, MFMA =
    2.5 PFLOP/s / train FLOP per sample (fwd + 2x for the backward)."""
    if args.model == "din":
        # fwd 51*2*4 + 51*2*16*2 + 8 ids/rows/len; bwd 408 + 2*3264
        nbytes = 3680 + 6936
        # attention unit [B*L, 4E = 128] -> 80 -> 40 -> 1 and top [B, 2E = 64] -> 200 -> 80 -> 1
        fwd = DIN_L * 2 * (128 * 80 + 80 * 40 + 40) + 2 * (64 * 200 + 200 * 80 + 80)
    else:
        fo = args.model == "deepfm"
        f, b = alg_bytes_per_sample(CRITEO_FIELDS, 16, CRITEO_DENSE, fo,
                                    4 if getattr(args, "table_dtype", "bf16") == "fp32" else 2)
        nbytes = f + b
        d0 = CRITEO_FIELDS * 16 + CRITEO_DENSE
        if fo:
            fwd = 2 * (d0 * 400 + 400 * 400 + 400 * 400 + 400)
        else:  # 3 cross layers d0 x d0 + deep 400-400 + Linear(400, 1) (stacked DCN-v2)
            fwd = 2 * (3 * d0 * d0 + d0 * 400 + 400 * 400 + 400)
    flops = 3 * fwd
    hbm = HBM_PEAK_GBS * 1e9 / nbytes
    mfma = MFMA_PEAK_TFLOPS * 1e12 / flops
    return {"samples_per_s_per_gpu": round(per_gpu_samples_s, 1),
            "alg_bytes_per_sample": nbytes, "train_flop_per_sample": flops,
            "hbm_roofline_samples_per_s": round(hbm, 1),
            "mfma_roofline_samples_per_s": round(mfma, 1),
            "frac_of_min_roofline": round(per_gpu_samples_s / min(hbm, mfma), 4)}


class _Ctx:
    """Stand-in autograd ctx for calling Function.forward directly."""
    def save_for_backward(self, *a):
        pass

    def set_materialize_grads(self, value):
        pass


# ----------------------------------------------------------------------------
# PCIe-inclusive rate: the same step fed from host memory by the columnar loader
# ----------------------------------------------------------------------------

def pcie_inclusive(step, args, sparse, dense_cols, label_col, device):
    """Train steps whose batches start in HOST memory: ``ColumnarLoader`` packs the
    epoch into pinned memory (outside the timed region, as a real epoch would be
    prepared ahead), then each batch crosses PCIe as one copy kernel reading the
    pinned record, on a branch of the step's HIP graph beside the step's kernels,
    ``depth - 1`` batches ahead (ColumnarLoader.capture_steps: one graph of
    ``depth`` steps, the record index a device cursor).  Reported beside ``value``
    (DESIGN.md §5), never as it."""
    from pytorchrec_amd.loader import ColumnarDataset, ColumnarLoader
    B = args.batch
    depth = 4
    n_batches = -(-max(args.steps, 12) // depth) * depth
    N = B * n_batches
    g = torch.Generator().manual_seed(7)
    cols = {c.feature_name: torch.randint(0, c.category_num, (N,), generator=g,
                                          dtype=torch.int32) for c in sparse}
    for c in dense_cols:
        cols[c.feature_name] = torch.rand(N, generator=g)
    cols[label_col.feature_name] = (torch.rand(N, generator=g) < 0.25).float()
    ds = ColumnarDataset(cols, dense_group=[c.feature_name for c in dense_cols])
    ld = ColumnarLoader(ds, B, device, depth=depth)
    for s, _ in ld.iter_slots():  # eager epoch: warms the model and fills every slot
        step(ld.slot_views(s))
    torch.cuda.synchronize()
    ge = ld.capture_steps(step)
    for _ in ge.replays():  # one untimed graph epoch
        pass
    ld.prepare_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in ge.replays():
        n += depth
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(n * B / el, 1), "unit": "samples/s", "steps": n,
            "ms_per_step": round(el / n * 1e3, 4), "h2d_bytes_per_step": ld.layout.record_bytes,
            "feed": f"ColumnarLoader (pytorchrec_amd/loader.py), depth {depth}: one packed pinned "
                    "record per batch read over PCIe by copy workgroups of the step's "
                    "mrec_tower_dw_ex launch (mrec_feed_job, a device cursor), depth - 1 "
                    "batches ahead; one graph of depth steps replayed (capture_steps)"}


# ----------------------------------------------------------------------------
# CPU baseline (oracle restatement of the reference path; rank 0, N = 1 only)
# ----------------------------------------------------------------------------

def host_cpu() -> dict:
    """The host's CPU (lscpu) and the share of it this process may use: the GPU box
    runs one job per GPU and gives it OMP_NUM_THREADS (16) of the host's cores."""
    info = {}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except (OSError, ValueError):
        pass
    def num(k):
        try:
            return int(info.get(k, ""))
        except ValueError:
            return None
    sockets, cps, tpc = num("Socket(s)"), num("Core(s) per socket"), num("Thread(s) per core")
    phys = sockets * cps if sockets and cps else None
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    return {"model": info.get("Model name"), "sockets": sockets, "cores_per_socket": cps,
            "threads_per_core": tpc, "physical_cores": phys, "affinity_cpus": affinity,
            "job_cpu_share": share,
            "threads_used": max(1, min(share, affinity, phys or affinity))}


def cpu_baseline(args):
    from oracle.models import RefDeepFM, criteo_batch, sgd_train_step
    cpu = host_cpu()
    threads = cpu["threads_used"]
    torch.set_num_threads(threads)
    nums = [args.rows_per_table] * CRITEO_FIELDS
    m = RefDeepFM(nums, CRITEO_DENSE, 16, (400, 400, 400))
    opt = torch.optim.SGD(m.parameters(), lr=args.lr)
    ids, dense, label = criteo_batch(nums, args.batch, seed=0, zipf=args.zipf)
    for _ in range(3):
        sgd_train_step(m, opt, ids, dense, label)
    ts, t_end = [], time.perf_counter() + args.cpu_seconds
    while (time.perf_counter() < t_end and len(ts) < 20) or len(ts) < 3:
        t = time.perf_counter()
        sgd_train_step(m, opt, ids, dense, label)
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    return {"value": round(args.batch / med, 1), "unit": "samples/s", "cores": threads,
            "kind": "port", "host_cpu": cpu,
            "sample": (f"{len(ts)} timed steps (median, after 3 warm-up) of the fp32 torch-CPU "
                       f"restatement of the reference path (26 nn.Embedding + 26 Embedding(rows,1), "
                       f"MLP 429-400-400-400-1, BCE, dense-grad SGD) at B={args.batch}, "
                       f"{args.rows_per_table} rows/table; {threads} threads = the job's CPU "
                       f"share (OMP_NUM_THREADS) of {cpu['physical_cores']} physical cores "
                       f"({cpu['sockets']} x {cpu['model']})"),
            "ms_per_step": round(med * 1e3, 3)}


# ----------------------------------------------------------------------------

def stub_main(args, json_out, world, rank):
    """--stub-step: the launcher and the max-over-ranks timing without a GPU (CPU
    tests): each step is one gloo all-reduce of a small tensor."""
    import torch.distributed as dist
    if os.environ.get("BENCH_STUB_FAIL_RANK") == str(rank):  # launcher test: a rank dies
        raise SystemExit(3)
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1024)

    def step():
        if world > 1:
            dist.all_reduce(t)
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el)
    if rank == 0:
        print(json.dumps({"metric": "launcher stub (gloo all-reduce per step, no GPU)",
                          "value": round(args.batch * world * args.steps / max(el, 1e-9), 1),
                          "unit": "samples/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "stub", "global_batch": args.batch * world,
                                     "rows_per_table": args.rows_per_table,
                                     "parallelism": f"gloo{world}"}}),
              file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        sys.exit(launch(args))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one "
                         f"process per GPU (bench.py --gpus N starts them itself)")
    # stdout carries exactly one JSON line: anything a native library prints there
    # (RCCL's version banner at communicator init) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub_step:
        return stub_main(args, json_out, world, rank)
    sharded = world > 1 or args.shard
    if args.same_gpu:
        if args.dist_backend != "gloo":
            raise SystemExit("bench.py: --same-gpu needs --dist-backend gloo")
        local = 0
    if args.dist_backend == "gloo":
        args.no_graph = True  # gloo collectives are host-driven: nothing to capture
    if world > 1 or args.force_collectives:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    comm = None
    if sharded:
        from pytorchrec_amd.sharding import ShardComm
        comm = ShardComm(force_collectives=args.force_collectives)
    builder = {"deepfm": build_deepfm, "dcnv2": build_dcnv2, "din": build_din}[args.model]
    model, sparse, dense_cols, label_col = builder(args, device, comm)
    from pytorchrec_amd.loss import BCEWithLogitsLoss
    model.compile(torch.optim.SGD(model.get_parameters(), lr=args.lr), BCEWithLogitsLoss(), [],
                  device)
    for bank in model.embedding_banks():
        bank.check_ids = False  # no host sync inside the captured step
    assert model.embeddings.update == "sgd", "SGD must fuse into the embedding backward"

    if args.model == "din":
        datas = [din_batch(args, 1000 * rank + s, device) for s in range(4)]
    else:
        bufs = [make_batch_buffer(args, sparse, 1000 * rank + s, device) for s in range(4)]
        datas = [batch_views(b, args, sparse, dense_cols, label_col) for b in bufs]

    def step(d):
        return model.train_step(d)["loss"]

    graphs = None
    if not args.no_graph:
        # one graph per resident batch (inputs used in place: no staging copy)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k in range(3):
                step(datas[k % 4])
        torch.cuda.current_stream().wait_stream(s)
        try:
            graphs = []
            for d in datas:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    step(d)
                graphs.append(g)
            multi = None
            G = max(1, min(args.graph_steps, 4))
            if G > 1:
                multi = torch.cuda.CUDAGraph()
                with torch.cuda.graph(multi, capture_error_mode="thread_local"):
                    for k in range(G):
                        step(datas[k])
        except Exception as e:  # e.g. a collective the runtime cannot capture
            print(f"bench: HIP graph capture failed ({type(e).__name__}: {e}); running eagerly",
                  file=sys.stderr, flush=True)
            args.no_graph = True
            torch.cuda.synchronize()
            graphs = None

    def run(i):
        if graphs is None:
            step(datas[i % 4])
        else:
            graphs[i % 4].replay()

    def run_steps(n):
        """n train steps, batch i % 4 at step i: G-step graphs while n allows, then
        single-step graphs (the G-step graph starts at batch 0: n is split so)."""
        i = 0
        if graphs is not None and multi is not None:
            while n - i >= G:
                multi.replay()
                i += G
        while i < n:
            run(i)
            i += 1

    if graphs is None:
        multi, G = None, 1
    run_steps(args.warmup)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    run_steps(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    from pytorchrec_amd.sharding import ShardedEmbeddingBank
    for b in model.embedding_banks():
        if isinstance(b, ShardedEmbeddingBank) and os.environ.get("MREC_BENCH_DIAG_NOCHECK") != "1":
            b.check_flags()  # an exchange overflow would make the run invalid: raise
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t)

    samples = args.batch * world * args.steps
    workloads = {
        "deepfm": "DeepFM Criteo-shaped (%s): 26 sparse x %d rows, D=16 bf16 tables with packed "
                  "first-order weight, 13 dense, MLP 400-400-400, BCE, SGD lr %g (fused "
                  "row-sparse update)%s" % (
                      "C5" if args.rows_per_table >= C5_ROWS else "C2", args.rows_per_table,
                      args.lr, ", tables row-sharded (id mod %d) over the ranks, RCCL "
                      "all-to-all" % world if sharded else ""),
        "dcnv2": "DCN-v2 Criteo-shaped (C3): 26 sparse x %d rows, D=16 bf16, 13 dense, 3 cross "
                 "layers 429x429, deep MLP 400-400, BCE, SGD lr %g" % (args.rows_per_table, args.lr),
        "din": "DIN Amazon-Electronics-shaped (C4): items 63,001(+PAD) / categories 801(+PAD), "
               "D=16 bf16, history L=50 (lengths U{1..50}), attention MLP 80-40-1, top MLP "
               "200-80-1, BCE, SGD lr %g" % args.lr,
    }
    metrics = {
        "deepfm": "samples/sec DeepFM Criteo-shaped batch 4096 at 1/2/4/8 MI355X; % HBM roofline",
        "dcnv2": "samples/sec DCN-v2 Criteo-shaped batch 4096, 3 cross layers, 1 MI355X",
        "din": "samples/sec DIN Amazon-Electronics-shaped batch 4096, L=50, 1 MI355X",
    }
    data_desc = ("synthetic (Amazon-Electronics-shaped: uniform ids seeds 0..3, U{1..50} history "
                 "lengths, Bernoulli(0.25) labels)" if args.model == "din" else
                 "synthetic (Criteo-shaped: uniform ids seed 0, U[0,1) dense, Bernoulli(0.25) "
                 "labels)" + (f", zipf {args.zipf}" if args.zipf else ""))
    result = {
        "metric": metrics[args.model],
        "value": round(samples / elapsed, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.table_dtype == "bf16" or args.model == "din" else
                 "bf16 tower, fp32 tables",
        "data": data_desc,
        "config": {"workload": workloads[args.model],
                   "global_batch": args.batch * world, "batch_per_gpu": args.batch,
                   "parallelism": (f"dp{world}+rowshard{world}" if sharded else "single"),
                   "collectives": (("gloo rehearsal, every rank on one GPU" if args.same_gpu
                                    else args.dist_backend) if world > 1 or
                                   args.force_collectives else None),
                   "exchange": (_exchange_desc(model, args) if sharded else None),
                   "hip_graph": not args.no_graph,
                   "steps_per_graph": G if graphs is not None else 0},
    }
    # what a PMC pass of this run stamps (tools/pmc_traffic.py reads it from the line)
    result["stamp"] = {"lib": lib_digest(), "workload": pmc_workload(args)}
    if (rank == 0 and not args.no_roofline and args.model == "deepfm" and sharded
            and graphs is not None and model.embeddings.use_compact(args.batch)):
        result.update(sharded_roofline(model, step, datas, args))
    elif rank == 0 and not args.no_roofline and args.model in ("deepfm", "dcnv2"):
        result.update(embedding_roofline(model, step, datas, args,
                                         in_step=graphs is not None and not sharded))
    if rank == 0 and not args.no_roofline and args.model == "din":
        ks = din_rooflines(model, datas[0], args)
        standalone = {k: v[0] for k, v in ks.items()}
        timing = ("standalone: the kernel launched alone, HIP events over back-to-back "
                  "graph replays")
        if graphs is not None:
            # in the graph-replayed train step, as C2 / C3 (the attention backward is
            # followed by the unclocked weight-gradient reduce: its waves' own span)
            t_in, _, _ = instep_kernel_times(step, datas, DIN_PAIR)
            if all(k in t_in for k in DIN_PAIR):
                ks = {k: (t_in[k],) + ks[k][1:] for k in ks}
                timing = ("in-step: the kernels' own clock (mrec_kernel_clock, s_memrealtime) "
                          "inside the graph-replayed train steps; mrec_din_att_fwd = its launch's "
                          "share of the step (first wave start to the tower's), mrec_din_att_bwd "
                          "= its waves' span (the unclocked weight-gradient reduce follows); "
                          "median over 4 steps x 30 replays")
        name = max(ks, key=lambda k: ks[k][0])  # the dominant kernel
        t, fl, nb = ks[name]
        ach = fl / t / 1e12
        traffic, tsrc = pmc_traffic([name], args)
        result["roofline"] = {"bound": "mfma", "kernel": name,
                              "achieved": round(ach, 2), "peak": MFMA_PEAK_TFLOPS,
                              "unit": "TFLOP/s", "frac": round(ach / MFMA_PEAK_TFLOPS, 4),
                              "traffic": traffic, "traffic_source": tsrc,
                              "avg_us": round(t * 1e6, 3), "timing": timing,
                              "standalone_us": round(standalone[name] * 1e6, 3),
                              "flop_per_launch": fl,
                              "flop_rule": "attention unit 2 L (128*80 + 80*40 + 40) per "
                                           "sample forward, x3 for the backward launch "
                                           "(forward recomputed)",
                              "hbm_GB/s": round(nb / t / 1e9, 1),
                              "hbm_frac": round(nb / t / 1e9 / HBM_PEAK_GBS, 4),
                              "alg_bytes_per_launch": nb}
        result["roofline_kernels"] = {k: {"avg_us": round(v[0] * 1e6, 3),
                                          "standalone_us": round(standalone[k] * 1e6, 3),
                                          "flop": v[1],
                                          "TFLOP/s": round(v[1] / v[0] / 1e12, 2),
                                          "bytes": v[2], "GB/s": round(v[2] / v[0] / 1e9, 1)}
                                      for k, v in ks.items()}
    if rank == 0:
        result["end_to_end"] = end_to_end(args, result["value"] / world)
    if (world == 1 and not sharded and not args.no_h2d and not args.no_graph
            and args.model == "deepfm"):
        result["pcie_inclusive"] = pcie_inclusive(step, args, sparse, dense_cols, label_col,
                                                  device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "deepfm":
        result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    # teardown: a HIP graph that captured RCCL work keeps a reference on the
    # communicator, and ncclCommDestroy waits for every such graph to be destroyed
    # (measured, tools/destroy_probe.py: destroy_process_group hangs while the graph
    # lives, returns in 0.4 s once it is released).  So every captured graph is
    # reset -- also any the gc still finds -- before the process group goes away.
    del run, run_steps
    graphs = multi = g = None
    n = release_graphs()
    if n:
        print(f"bench: reset {n} HIP graph(s) still reachable at teardown", file=sys.stderr,
              flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


def _exchange_desc(model, args):
    """The row-sharded exchange the bank ran and its bytes per rank and direction
    (rows forward / gradients backward; ids are 4 B per slot)."""
    b = model.embeddings
    compact = b.use_compact(args.batch)
    W = b.world
    if compact:
        per = b.cap_rows * b.wire_bytes()
        return {"kind": "compact (one record per distinct id)", "cap": b.cap,
                "cap_rows": b.cap_rows, "record_bytes": b.wire_bytes(),
                "bytes_per_rank_each_way": W * per, "remote_bytes_each_way": (W - 1) * per}
    rows = W * b.n_tables * b.cap
    return {"kind": "slot (one row per lookup)", "cap": b.cap,
            "bytes_rows_fwd": rows * b.row_stride * b.weight.element_size(),
            "bytes_grads_bwd": rows * b.g_ld * 4}


def release_graphs() -> int:
    """Reset every torch CUDAGraph the garbage collector can still reach (their
    captured RCCL plans hold the communicator), then drain the device."""
    import gc
    gc.collect()
    live = [o for o in gc.get_objects() if isinstance(o, torch.cuda.CUDAGraph)]
    for gr in live:
        gr.reset()
    n = len(live)
    del live
    torch.cuda.synchronize()
    return n

if __name__ == "__main__":
    main()
