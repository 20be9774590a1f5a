"""Per-kernel averages of rocprofv3 --pmc counter CSVs (k_counter_collection.csv)."""
import collections
import csv
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0][-60:]
            grid = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
            agg[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in sorted(agg.items(), key=lambda kv: kv[0][1]):
        if len(next(iter(cs.values()))) < 5:
            continue
        print(f"{name} blocks={grid}")
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v) / len(v):14.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
