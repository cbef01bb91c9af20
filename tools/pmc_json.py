"""Merge a FETCH_SIZE pass and a WRITE_SIZE pass (rocprofv3 --pmc counter
collection CSVs) into the per-kernel summary bench.py reads (profiles/rNN_pmc.json).
FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  Two read figures per kernel:
fetch_size_kib as counted, and fetch_bytes = 2 x FETCH_SIZE (the guide's gfx950
correction for wide, 16-B-per-lane coalesced reads, MI355X_MICROARCH.md HBM
section).  bench.py's roofline `traffic` uses the raw count (fetch_size_kib *
1024 + write_bytes): the path's kernels load <= 4 B per lane, for which the x2
does not apply."""
import collections
import csv
import json
import sys


def means(path, counter):
    d = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            d[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: (len(v), sum(v) / len(v)) for k, v in d.items()}


fetch, write = means(sys.argv[1], "FETCH_SIZE"), means(sys.argv[2], "WRITE_SIZE")
out = {"note": sys.argv[4] if len(sys.argv) > 4 else "", "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    e = {}
    if k in fetch:
        e.update(launches_fetch_pass=fetch[k][0], fetch_size_kib=fetch[k][1], fetch_bytes=fetch[k][1] * 1024 * 2)
    if k in write:
        e.update(launches_write_pass=write[k][0], write_size_kib=write[k][1], write_bytes=write[k][1] * 1024)
    out["kernels"][k] = e
json.dump(out, open(sys.argv[3], "w"), indent=1)
