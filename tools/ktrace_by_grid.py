#!/usr/bin/env python3
"""Kernel durations per (kernel, grid size) from a rocprofv3 --kernel-trace csv
(<prefix>_kernel_trace.csv): count, mean / min / max / median duration in us.
A kernel launched at several sizes (the pyramid build at 1080p in the loop, at
4K in the bench's 4K leg) gets one entry per grid, so a roofline can use the
kernel time of its own launches (rocprof's GPU start/end, no launch cost).

    python tools/ktrace_by_grid.py <kernel_trace.csv> <out.json> [note] [kernel substr ...]
"""
import collections
import csv
import json
import statistics
import sys


def kernel_key(name: str) -> str:
    """The demangled name without its parameter list ("(anonymous namespace)::"
    dropped first, so that its parenthesis does not end the name)."""
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def summarize(path, substrs=()):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if substrs and not any(s in name for s in substrs):
            continue
        g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)
        per[(kernel_key(name), g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    out = []
    for (name, g), d in sorted(per.items()):
        out.append({"kernel": name, "grid": g, "dispatches": len(d), "avg_us": round(sum(d) / len(d), 3),
                    "median_us": round(statistics.median(d), 3), "min_us": round(min(d), 3),
                    "max_us": round(max(d), 3)})
    return out


def main():
    path, dst = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = summarize(path, sys.argv[4:])
    json.dump({"note": note, "source": path.split("/")[-1], "entries": rows}, open(dst, "w"), indent=1)
    for r in rows:
        print(f'{r["kernel"][:60]:60s} grid {r["grid"]:>10d} n {r["dispatches"]:6d} avg {r["avg_us"]:9.2f} us')


if __name__ == "__main__":
    main()
