"""Per-launch median durations of the steady-state step from a rocprofv3 kernel trace.

usage: python tools/trace_steps.py <k_kernel_trace.csv> [last_n_launches]
Groups the trace's kernels by (name, grid) and prints median / count, plus the
median gap between consecutive kernels (the hipGraph node boundary)."""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
by = {}
for r in tail:
    wgs = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])) * int(r.get("Grid_Size_Y") or 1) * \
        int(r.get("Grid_Size_Z") or 1)
    key = (r["Kernel_Name"][:70], wgs)
    by.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0.0
for (name, wgs), v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    med = st.median(v) / 1000
    print(f"{med:8.2f} us  x{len(v):5d}  {wgs:6d} WGs  {name}")
gaps = [int(tail[i + 1]["Start_Timestamp"]) - int(tail[i]["End_Timestamp"]) for i in range(len(tail) - 1)]
print(f"median gap {st.median(gaps) / 1000:.2f} us")
