"""Print a rocprofv3 kernel_stats.csv as 'total  calls  avg  pct  name' lines."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e3:10.1f}us {int(r['Calls']):5d} avg {float(r['AverageNs']) / 1e3:8.2f}us "
          f"{100 * t / tot:5.1f}%  {r['Name'][:110]}")
print(f"total us {tot / 1e3:.1f}")
