"""Summarise a rocprofv3 --kernel-trace --stats kernel_stats.csv (top kernels)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs'])/1e3:9.1f}us {int(r['Calls']):5d} avg "
          f"{float(r['AverageNs'])/1e3:7.2f}us {float(r['Percentage']):5.1f}%  {r['Name'][:100]}")
print("total us", round(tot / 1e3, 1))
