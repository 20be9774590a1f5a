#!/usr/bin/env python
"""Per-kernel summary (calls, total / mean / min / max us, share) of a rocprofv3
``--kernel-trace`` database (rocpd SQLite, the ROCm 7 default output format).

Usage: python tools/rocpd_summary.py gpurun_out/prof/run_results.db [out.csv] [--top N]
"""
import csv
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = []
    for name, n, tot, mn, mx in rows:
        out.append({"kernel": name if len(name) < 160 else name[:157] + "...", "calls": n,
                    "total_us": round(tot / 1e3, 3), "mean_us": round(tot / n / 1e3, 3),
                    "min_us": round(mn / 1e3, 3), "max_us": round(mx / 1e3, 3),
                    "pct": round(100.0 * tot / total, 2)})
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 25
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    rows = summary(args[0])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)
    for r in rows[:top]:
        print(f"{r['pct']:6.2f}% {r['calls']:6d} x {r['mean_us']:10.3f} us  {r['kernel'][:110]}")


if __name__ == "__main__":
    main()
