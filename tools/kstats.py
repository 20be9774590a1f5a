"""Print the top kernels of a rocprofv3 kernel_stats.csv: name, calls, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Percentage"][:5])
