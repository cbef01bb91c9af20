"""Per-kernel mean of every counter over the given rocprofv3 counter_collection CSVs."""
import collections
import csv
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        d[row["Kernel_Name"][:70]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, ctr in d.items():
    print(k)
    for c, v in sorted(ctr.items()):
        print(f"    {c:28s} n={len(v):4d} mean={sum(v) / len(v):16.1f}")
