"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into per-kernel HBM bytes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir>  > profiles/pmc_traffic.json

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE counts
half the bytes of a wide coalesced *streaming* read on gfx950 and is uncalibrated
for other widths.  The embedding kernels' reads are dominated by random 64-B row
requests; calibrated on mrec_interact_fwd (known read bytes: 4096 x 26 full 64-B
rows + ids + dense = 7.5 MB vs FETCH_SIZE 8.4 MiB undoubled, and WRITE_SIZE = the
3.8 MB of x0 / fm_sum / logit exactly) those requests count 1:1, so
hbm_bytes = FETCH_SIZE + WRITE_SIZE (the doubled figure is kept as an upper bound).
Infinity-Cache hits are counted, so this is memory-side (L2-miss) traffic: an
upper bound on the HBM bytes.
"""
import collections
import csv
import glob
import json
import os
import sys

# substring of the kernel name -> key (first match wins)
KERNELS = {"interact_plan_kernel": "mrec_interact_fwd_ex", "interact_kernel": "mrec_interact_fwd",
           "plan_hash_kernel": "mrec_emb_bwd_plan", "plan_kernel": "mrec_emb_bwd_plan",
           "apply_kernel": "mrec_emb_bwd_apply", "gemm_dma_kernel": "mrec_gemm",
           "gemm_multi_kernel": "mrec_gemm_multi", "gather_kernel": "mrec_emb_gather_fwd"}


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for k, v in KERNELS.items():
            if k in name:
                agg[v].append(float(r["Counter_Value"]))
                break
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                     "bench.py --steps 5 --warmup 3; hbm_bytes = (FETCH_SIZE + WRITE_SIZE) * 1024 "
                     "(random 64-B row reads count 1:1, calibrated on mrec_interact_fwd); "
                     "upper_bound uses 2*FETCH_SIZE (the streaming-read correction)",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        out["kernels"][k] = {"fetch_kib_avg": round(fetch[k], 1), "write_kib_avg": round(write[k], 1),
                             "dispatches": nf[k],
                             "hbm_bytes_per_launch": int((fetch[k] + write[k]) * 1024),
                             "upper_bound_bytes": int((2 * fetch[k] + write[k]) * 1024)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
