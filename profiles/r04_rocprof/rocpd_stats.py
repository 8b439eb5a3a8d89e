"""Kernel statistics from a rocprofv3 SQLite (rocpd) database -- this ROCm's rocprofv3 writes
`<name>_results.db` unless told otherwise: python tools/rocpd_stats.py DB [out.csv] [top]
Prints (and optionally writes as CSV) per-kernel calls, total / mean / min / max microseconds and the
share of summed kernel time, names shortened to 140 characters."""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), min(duration), max(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = []
    for name, n, s, lo, hi in rows:
        out.append({"kernel": name[:140], "calls": n, "total_us": round(s / 1e3, 1), "mean_us": round(s / n / 1e3, 2),
                    "min_us": round(lo / 1e3, 2), "max_us": round(hi / 1e3, 2), "pct": round(100.0 * s / tot, 2)})
    return out


def main():
    db = sys.argv[1]
    rows = stats(db)
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    for r in rows[:top]:
        print("%7.2f%% %6d calls %12.1f us  mean %10.2f  %s" % (r["pct"], r["calls"], r["total_us"], r["mean_us"],
                                                           r["kernel"][:100]))


if __name__ == "__main__":
    main()
