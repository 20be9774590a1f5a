"""Summarise a rocprofv3 kernel trace (CSV) into a markdown table.

usage: python tools/prof_summary.py <kernel_trace.csv> [--title T] [--skip N] > profiles/x.md
Groups dispatches by (kernel, grid), reports count / mean / p50 / total time,
and the mean gap between consecutive dispatches on the same queue.
"""
import argparse
import collections
import csv
import statistics


def short(name):
    name = name.split("(")[0]
    for pre in ("void ", "ea::"):
        name = name.replace(pre, "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--title", default="kernel trace summary")
    ap.add_argument("--skip", type=int, default=0, help="skip the first N dispatches (warmup/capture)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[a.skip:]
    groups = collections.OrderedDict()
    gaps = []
    prev_end = {}
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r["Queue_Id"]
        if q in prev_end and 0 <= s - prev_end[q] < 50_000:
            gaps.append(s - prev_end[q])
        prev_end[q] = e
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        key = (short(r["Kernel_Name"]), grid, r["LDS_Block_Size"], r["VGPR_Count"], r["Scratch_Size"])
        groups.setdefault(key, []).append((e - s) / 1000.0)
    total = sum(sum(v) for v in groups.values())
    print(f"# {a.title}\n")
    print(f"{len(rows)} dispatches, total kernel time {total/1000:.2f} ms; "
          f"median inter-dispatch gap {statistics.median(gaps)/1000 if gaps else 0:.2f} us\n")
    print("| kernel | blocks | LDS B | VGPR | scratch | count | mean us | p50 us | total % |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for (k, grid, lds, vgpr, scr), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{k}` | {grid} | {lds} | {vgpr} | {scr} | {len(v)} | {statistics.mean(v):.2f} | "
              f"{statistics.median(v):.2f} | {100*sum(v)/total:.1f} |")


if __name__ == "__main__":
    main()
