"""One replayed step's kernel sequence from a rocprofv3 --kernel-trace csv:
    python tools/step_sequence.py <run_kernel_trace.csv> [anchor substring]
Prints, for the median-length stretch between consecutive launches of the anchor
kernel (default: the fused tower), each kernel's gap before it and its duration."""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "tower_kernel<8, false"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    spans = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1)]
    spans = [s for s in spans if s[1] - s[0] < 64]
    if not spans:
        raise SystemExit("no anchor stretch")
    lens = sorted(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) for a, b in spans)
    med = lens[len(lens) // 2]
    a, b = next(s for s in spans if int(rows[s[1]]["Start_Timestamp"]) - int(rows[s[0]]["Start_Timestamp"]) == med)
    prev_end = None
    tot = 0.0
    for r in rows[a:b]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = 0.0 if prev_end is None else (st - prev_end) / 1e3
        tot += (en - st) / 1e3
        print(f"{gap:7.2f} {(en - st) / 1e3:7.2f}  {r['Kernel_Name'][:110]}")
        prev_end = en
    print(f"sum of kernel durations {tot:.1f} us; anchor to next anchor {med / 1e3:.1f} us")


if __name__ == "__main__":
    main()
