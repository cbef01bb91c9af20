"""Per-dispatch PMC values of one kernel grouped by grid size (rocprofv3
--pmc csv): the mean of every counter over the dispatches of each grid, so a
multi-level kernel's levels can be told apart.  Usage:
    python tools/pmc_by_grid.py <pmc_counter_collection.csv> <kernel substring>"""
import collections
import csv
import sys


def main(path, kern):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    grid = {}
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        grid[d] = int(r["Grid_Size"])
    by = collections.defaultdict(list)
    for d, cs in per.items():
        by[grid[d]].append(cs)
    for g in sorted(by, reverse=True):
        ds = by[g]
        names = sorted({n for cs in ds for n in cs})
        vals = {n: sum(cs.get(n, 0.0) for cs in ds) / len(ds) for n in names}
        print(f"grid {g:>10d}  dispatches {len(ds)}")
        for n in names:
            print(f"    {n:28s} {vals[n]:16.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
