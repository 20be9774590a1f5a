#!/usr/bin/env python
"""Concurrency of the kernels in a rocprofv3 --kernel-trace database: per queue and
stream the kernel count and busy time, and over the whole trace the sum of kernel
durations vs the length of their union (sum / union > 1 means kernels overlapped).
Usage: python tools/rocpd_overlap.py run_results.db [name-substring]
       python tools/rocpd_overlap.py run_results.db --copies   (copy / kernel overlap)"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = c.execute("select start, end, queue_id, stream_id, name from kernels order by start").fetchall()
    rows = [r for r in rows if sub in r[4]]
    if not rows:
        print("no kernels")
        return
    per = {}
    for s, e, q, st, _ in rows:
        k = (q, st)
        n, busy = per.get(k, (0, 0))
        per[k] = (n + 1, busy + (e - s))
    for (q, st), (n, busy) in sorted(per.items()):
        print(f"queue {q} stream {st}: {n} kernels, busy {busy / 1e6:.3f} ms")
    total = sum(e - s for s, e, *_ in rows)
    union, cur_s, cur_e = 0, None, None
    events = []
    for s, e, *_ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        events += [(s, 1), (e, -1)]
    union += cur_e - cur_s
    events.sort()
    depth, peak, hist = 0, 0, {}
    last = events[0][0]
    for t, d in events:
        hist[depth] = hist.get(depth, 0) + (t - last)
        depth += d
        peak = max(peak, depth)
        last = t
    span = rows[-1][1] - rows[0][0]
    print(f"kernels {len(rows)}; sum of durations {total / 1e6:.3f} ms; union {union / 1e6:.3f} ms; "
          f"span {span / 1e6:.3f} ms; mean concurrency while busy {total / max(union, 1):.2f}; peak {peak}")
    print("time at concurrency depth (ms): " +
          ", ".join(f"{d}: {v / 1e6:.3f}" for d, v in sorted(hist.items()) if v > 0))


if __name__ == "__main__" and "--copies" not in sys.argv:
    main()


def copy_kernel_overlap(db):
    """Memory copies vs kernels (a --memory-copy-trace run): bytes, copy time, and how much
    of the copy time ran while at least one kernel was running."""
    c = sqlite3.connect(db)
    ks = c.execute("select start, end from kernels order by start").fetchall()
    cs = c.execute("select start, end, size from memory_copies order by start").fetchall()
    # merge kernel intervals
    merged = []
    for s, e in ks:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    import bisect
    starts = [m[0] for m in merged]
    tot = ov = nbytes = 0
    for s, e, n in cs:
        tot += e - s
        nbytes += n
        i = max(0, bisect.bisect_right(starts, s) - 1)
        while i < len(merged) and merged[i][0] < e:
            ov += max(0, min(e, merged[i][1]) - max(s, merged[i][0]))
            i += 1
    print(f"copies {len(cs)}: {nbytes / 1e9:.3f} GB in {tot / 1e6:.3f} ms ({nbytes / max(tot, 1):.1f} GB/s while "
          f"copying); {100.0 * ov / max(tot, 1):.1f} % of copy time overlapped kernels; kernels busy "
          f"{sum(e - s for s, e in merged) / 1e6:.3f} ms")


if __name__ == "__main__" and "--copies" in sys.argv:
    copy_kernel_overlap(sys.argv[1])
