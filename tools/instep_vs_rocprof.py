"""Compare bench.py's in-step kernel times (the kernel clock, roofline_kernels) with
rocprofv3's per-kernel averages of the PRODUCTION instantiations (template flag
KC = false) from a `rocprofv3 --kernel-trace --stats --output-format csv` run of
the same bench command.

  python tools/instep_vs_rocprof.py BENCH.json KERNEL_STATS.csv"""
import csv
import json
import sys

KERNELS = {"interact_plan_kernel": "mrec_interact_fwd_ex",
           "apply_hash_kernel": "mrec_emb_bwd_apply_ex",
           "tower_kernel": "mrec_tower_fwd_bwd",
           "tower_dw_kernel": "mrec_tower_dw_ex"}


def main(bench_json, stats_csv):
    line = [ln for ln in open(bench_json).read().splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    rk = d["roofline_kernels"]
    tot_r = tot_c = 0.0
    for r in csv.DictReader(open(stats_csv)):
        for k, entry in KERNELS.items():
            if f"::{k}<" in r["Name"] and "false>(" in r["Name"] and entry in rk:
                a = float(r["AverageNs"]) / 1000
                c = rk[entry]["avg_us"]
                tot_r += a
                tot_c += c
                print(f"{entry:24s} rocprof {a:7.2f} us  in-step clock {c:7.2f} us  "
                      f"({100 * (c - a) / a:+.1f}%)  rocprof calls {r['Calls']}")
    print(f"{'sum':24s} rocprof {tot_r:7.2f} us  in-step clock {tot_c:7.2f} us  "
          f"({100 * (tot_c - tot_r) / tot_r:+.1f}%)   bench ms_per_step {d['ms_per_step']}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
