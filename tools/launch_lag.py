#!/usr/bin/env python3
"""Launch-to-start lag per kernel from a `rocprofv3 --kernel-trace
--hip-runtime-trace --output-format csv` run: each dispatch is matched to the
HIP call that enqueued it (Correlation_Id); lag = the kernel's GPU start minus
the end of that call.  Prints median / p10 / p90 per (kernel, queue), and the
host gap between consecutive launches of the loop's step.

usage: tools/launch_lag.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [--skip N]
"""
import argparse
import csv
import glob
import os
import re
import statistics
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("tbdk::", "").replace("void ", "")
    return n[:34]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=200, help="dispatches to skip (set-up, warm-up)")
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    at = glob.glob(os.path.join(a.dir, "**", "*hip_api_trace.csv"), recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(at)):
        api[r["Correlation_Id"]] = (r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))[a.skip:]
    lag = defaultdict(list)
    for r in ks:
        c = api.get(r["Correlation_Id"])
        if not c:
            continue
        lag[(short(r["Kernel_Name"]), r["Queue_Id"])].append((int(r["Start_Timestamp"]) - c[2]) / 1e3)
    print(f"{'kernel':34s} {'queue':>5s} {'n':>6s} {'lag p10':>8s} {'median':>8s} {'p90':>8s} us")
    for (k, q), v in sorted(lag.items(), key=lambda kv: -len(kv[1])):
        v.sort()
        print(f"{k:34s} {q:>5s} {len(v):6d} {v[len(v) // 10]:8.1f} {statistics.median(v):8.1f} "
              f"{v[(9 * len(v)) // 10]:8.1f}")


if __name__ == "__main__":
    main()
