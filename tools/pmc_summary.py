"""Per-kernel median of one PMC counter from a rocprofv3 --pmc counter_collection.csv
(KiB per dispatch, summed over the counter's instances): the summaries kept under
profiles/<round>/pmc/."""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, counter):
    per = defaultdict(float)  # (dispatch, kernel) -> value
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[(r["Dispatch_Id"], r["Kernel_Name"])] += float(r["Counter_Value"])
    by_k = defaultdict(list)
    for (_, k), v in per.items():
        by_k[k.split("(")[0]].append(v)
    rows = sorted(by_k.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1]))
    for k, vs in rows[:12]:
        print(f"{k[:80]:80s} n={len(vs):4d} median={statistics.median(vs):12.1f} KiB "
              f"min={min(vs):12.1f} max={max(vs):12.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
