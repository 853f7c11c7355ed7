"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into per-kernel
HBM bytes, stamped with the run they came from (profiles/pmc_traffic.json, read
by bench.py for roofline.traffic).

    python tools/pmc_traffic.py <out.json> <fetch_dir> <write_dir> [<fetch_dir> <write_dir> ...]

Each pair is one bench.py workload profiled twice (the two counters do not fit one
TCC pass).  The workload key and the library digest come from the bench line the
FETCH pass printed (``stamp``: model, batch, rows per table, Zipf alpha, sharding /
exchange; the source digest libmrec.so was built from): bench.py reports the traffic
only for a run with its own workload and library.  A stamp for the same workload
replaces the older one in <out.json>; others are kept.

Calibration (tools/micro/ceilings.hip under --pmc, profiles/r02/pmc_calibration.json):
FETCH_SIZE counts every memory-side read request as 64 B -- a 2 GiB streaming copy
reads as 1 GiB (its 128-B requests tallied at 64 B, MI355X_MICROARCH.md §HBM), and
random 32-, 64- and 128-B rows all read as 64 B per row.  WRITE_SIZE is exact for
16-B-per-lane stores.  The embedding kernels' reads are dominated by random 64-B
row requests (counted exactly), their streaming reads (ids, dx) count half, so
    hbm_bytes_per_launch = (FETCH_SIZE + WRITE_SIZE) * 1024   (the estimate)
    upper_bytes          = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (every read a 128-B one)
Infinity-Cache hits are counted, so both are memory-side (L2-miss) traffic.
"""
import collections
import csv
import datetime
import glob
import json
import os
import re
import subprocess
import sys

# substring of the kernel name -> bench.py roofline key (first match wins)
KERNELS = {"din_att_bwd": "mrec_din_att_bwd", "din_att_fwd": "mrec_din_att_fwd",
           "bk_apply_kernel": "mrec_emb_bwd_large_fused",
           "interact_plan_kernel": "mrec_interact_fwd_ex", "interact_rec_kernel": "mrec_interact_fwd_ex",
           "interact_kernel": "mrec_interact_fwd",
           "plan_hash_kernel": "mrec_emb_bwd_plan", "apply_hash_kernel": "mrec_emb_bwd_apply",
           "apply_kernel": "mrec_emb_bwd_apply", "tower_dw_kernel": "mrec_tower_dw_ex",
           "tower_kernel": "mrec_tower_fwd_bwd", "gemm_dma_kernel": "mrec_gemm",
           "gemm_multi_kernel": "mrec_gemm_multi", "gather_kernel": "mrec_emb_gather_fwd",
           "bucketize_dedup_kernel": "mrec_shard_bucketize_dedup",
           "gather_wire_kernel": "mrec_shard_gather_wire", "wire_move_kernel": "mrec_shard_wire_move",
           "sgd_multi_kernel": "mrec_sgd_multi"}

# the kernel clock's instantiations (template flag KC = true: the last template
# argument, the second of the tower kernels'; wire_move<true, true> is the slot
# exchange's fp32 unpack, not clocked and not on the compact path) run only in
# bench.py's in-step timing graphs
_CLOCKED = re.compile(r"(interact_plan_kernel|interact_rec_kernel|apply_hash_kernel|"
                      r"bucketize_dedup_kernel|gather_wire_kernel|wire_move_kernel|sgd_multi_kernel|"
                      r"din_att_bwd2_kernel|din_att_fwd_wave_kernel)<[^()]*true>\(|"
                      r"(tower_kernel|tower_dw_kernel)<\d+, true")  # (KC second: <PF, KC, CROSS / FEED>)


def per_kernel(d, counter):
    """Per bench key: the median over the run's production dispatches of the summed
    counter (the sharded step has two apply dispatches per step, sender and owner: the
    median of each kind, summed -- kinds told apart by their kernel names)."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or _CLOCKED.search(r["Kernel_Name"]):
            continue
        for k, v in KERNELS.items():
            if k in r["Kernel_Name"]:
                agg[v][r["Kernel_Name"]].append(float(r["Counter_Value"]))
                break
    med = {k: sum(sorted(x)[len(x) // 2] for x in by_name.values()) for k, by_name in agg.items()}
    cnt = {k: sum(len(x) for x in by_name.values()) for k, by_name in agg.items()}
    return med, cnt


def bench_stamp(d):
    """The ``stamp`` of the bench line printed by the run profiled into ``d`` (its log
    sits beside it: <d>.log)."""
    for line in open(d.rstrip("/") + ".log"):
        line = line.strip()
        if line.startswith("{") and '"stamp"' in line:
            return json.loads(line)["stamp"]
    raise SystemExit(f"no bench line with a stamp in {d}.log")


def main():
    out_path, rest = sys.argv[1], sys.argv[2:]
    commit = os.environ.get("MREC_COMMIT")  # the GPU box has no .git: passed in by the caller
    if not commit:
        try:
            commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip() or None
        except OSError:
            commit = None
    try:
        doc = json.load(open(out_path))
        if not isinstance(doc.get("runs"), list) or not all("workload" in r for r in doc["runs"]):
            doc = {}
    except (OSError, ValueError):
        doc = {}
    doc["source"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                     "bench.py --steps 5 --warmup 3 (tools/gpu_pmc.sh); per-kernel median over "
                     "production dispatches (clocked instantiations excluded)")
    doc["correction"] = ("hbm_bytes = (FETCH_SIZE + WRITE_SIZE) KiB (random 64-B row reads "
                         "count 1:1, calibrated: profiles/r02/pmc_calibration.json); "
                         "upper_bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB")
    runs = doc.get("runs", [])
    while rest:
        fdir, wdir = rest[:2]
        rest = rest[2:]
        st_f, st_w = bench_stamp(fdir), bench_stamp(wdir)
        if st_f != st_w:
            raise SystemExit(f"{fdir} and {wdir} profiled different runs: {st_f} / {st_w}")
        fetch, nf = per_kernel(fdir, "FETCH_SIZE")
        write, _ = per_kernel(wdir, "WRITE_SIZE")
        kernels = {
            k: {"fetch_kib": round(fetch[k], 1), "write_kib": round(write[k], 1),
                "dispatches": nf[k], "hbm_bytes_per_launch": int((fetch[k] + write[k]) * 1024),
                "upper_bytes": int((2 * fetch[k] + write[k]) * 1024)}
            for k in sorted(set(fetch) & set(write))}
        run = {"workload": st_f["workload"], "lib": st_f["lib"], "commit": commit,
               "utc": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ"),
               "kernels": kernels}
        runs = [r for r in runs if r["workload"] != run["workload"]] + [run]
    doc["runs"] = runs
    with open(out_path, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({"runs": [(r["workload"], r["lib"][:12] if r["lib"] else None) for r in runs]}))


if __name__ == "__main__":
    main()
