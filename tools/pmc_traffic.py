"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into per-kernel
HBM bytes, stamped with the run they came from (profiles/pmc_traffic.json, read
by bench.py for roofline.traffic).

    python tools/pmc_traffic.py <out.json> <model> <batch> <rows> <fetch_dir> <write_dir> [...]

(several models: repeat the <model> <batch> <rows> <fetch_dir> <write_dir> group)

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
           "bk_apply_kernel": "mrec_emb_bwd_large_fused", "interact_plan_kernel": "mrec_interact_fwd_ex", "interact_kernel": "mrec_interact_fwd",
           "plan_hash_kernel": "mrec_emb_bwd_plan", "apply_hash_kernel": "mrec_emb_bwd_apply",
           "apply_kernel": "mrec_emb_bwd_apply", "tower_kernel": "mrec_tower_fwd_bwd",
           "gemm_dma_kernel": "mrec_gemm", "gemm_multi_kernel": "mrec_gemm_multi",
           "gather_kernel": "mrec_emb_gather_fwd"}


# the kernel clock's instantiations (template flag KC = true, the last template
# argument) run only in bench.py's in-step timing graphs: not the product kernels
_CLOCKED = re.compile(r"(interact_plan_kernel|apply_hash_kernel|tower_kernel|tower_dw_kernel)<[^()]*true>\(")


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or _CLOCKED.search(r["Kernel_Name"]):
            continue
        for k, v in KERNELS.items():
            if k in r["Kernel_Name"]:
                agg[v].append(float(r["Counter_Value"]))
                break
    # the median dispatch (the roofline timing launches dominate the count)
    return ({k: sorted(v)[len(v) // 2] for k, v in agg.items()}, {k: len(v) for k, v in agg.items()})


def main():
    out_path, rest = sys.argv[1], sys.argv[2:]
    commit = os.environ.get("MREC_COMMIT")  # the GPU box has no .git: passed in by the caller
    if not commit:
        try:
            commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip() or None
        except OSError:
            commit = None
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                     "bench.py --steps 5 --warmup 3 (tools/gpu_pmc.sh); per-kernel median over "
                     "dispatches",
           "correction": "hbm_bytes = (FETCH_SIZE + WRITE_SIZE) KiB (random 64-B row reads "
                         "count 1:1, calibrated: profiles/r02/pmc_calibration.json); "
                         "upper_bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB",
           "run": None, "kernels": {}}
    while rest:
        model, batch, rows, fdir, wdir = rest[:5]
        rest = rest[5:]
        fetch, nf = per_kernel(fdir, "FETCH_SIZE")
        write, _ = per_kernel(wdir, "WRITE_SIZE")
        doc["kernels"][model] = {
            k: {"fetch_kib": round(fetch[k], 1), "write_kib": round(write[k], 1),
                "dispatches": nf[k], "hbm_bytes_per_launch": int((fetch[k] + write[k]) * 1024),
                "upper_bytes": int((2 * fetch[k] + write[k]) * 1024)}
            for k in sorted(set(fetch) & set(write))}
        run = {"model": model, "batch": int(batch), "rows_per_table": int(rows), "commit": commit,
               "utc": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ")}
        doc.setdefault("runs", []).append(run)
    # bench.py matches `run` against its own workload: the stamp of the first model
    # (deepfm), the rest under "runs"
    doc["run"] = doc["runs"][0]
    with open(out_path, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
