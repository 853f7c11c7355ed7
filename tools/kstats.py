"""Per-kernel summary (calls, total / average / min / max us) from a rocprofv3
results database (rocpd sqlite: the default output of `rocprofv3 --kernel-trace`
on this image).  Usage: python tools/kstats.py <run_results.db> [top N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    c = sqlite3.connect(db)
    rows = c.execute(
        "select ks.display_name, count(*), sum(k.end - k.start), avg(k.end - k.start), "
        "min(k.end - k.start), max(k.end - k.start) from rocpd_kernel_dispatch k "
        "join rocpd_info_kernel_symbol ks on k.kernel_id = ks.id group by ks.display_name "
        "order by sum(k.end - k.start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} "
          f"{'max_us':>9s} {'pct':>6s}")
    for name, n, s, a, mn, mx in rows[:top]:
        short = name if len(name) <= 70 else name[:67] + "..."
        print(f"{short:70s} {n:6d} {s / 1e3:10.2f} {a / 1e3:9.3f} {mn / 1e3:9.3f} {mx / 1e3:9.3f} "
              f"{100 * s / tot:6.2f}")


if __name__ == "__main__":
    main()
