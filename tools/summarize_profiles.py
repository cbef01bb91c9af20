#!/usr/bin/env python3
"""Turn a tools/profile_round.sh run (gpurun_out/prof_<tag>/) into the committed
profiles/<tag>_* files:

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the default bench
  <tag>_bench.json         the bench JSON line printed under that profiler run
  <tag>_pmc.json           per-kernel mean FETCH_SIZE / WRITE_SIZE per launch (separate
                           --pmc passes), raw and as bytes; FETCH_SIZE is doubled per the
                           gfx950 note in MI355X_MICROARCH.md (HBM section)
"""
import collections
import csv
import json
import os
import shutil
import sys


def pmc(path):
    d = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        d[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: (len(v), sum(v) / len(v)) for k, v in d.items()}


def main(tag="r01"):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "bench_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    lines = [l for l in open(os.path.join(src, "bench.json")) if l.startswith("{")]
    open(os.path.join(dst, f"{tag}_bench.json"), "w").write(lines[-1])
    fetch = pmc(os.path.join(src, "fetch", "bench_counter_collection.csv"))
    write = pmc(os.path.join(src, "write", "bench_counter_collection.csv"))
    out = {"note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (kernel trace only), "
                   "bench.py --steps 60 --no-cpu-baseline; values are per-launch means. FETCH_SIZE/WRITE_SIZE "
                   "are KiB; fetch_bytes doubles FETCH_SIZE (gfx950 reports 1/2 of wide coalesced reads, "
                   "MI355X_MICROARCH.md HBM section; other access widths uncalibrated); Infinity-Cache hits "
                   "are included in these memory-side counters.",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, None))
        nw, w = write.get(k, (0, None))
        out["kernels"][k] = {"launches_fetch_pass": nf, "fetch_size_kib": f, "fetch_bytes": None if f is None else 2 * f * 1024,
                             "launches_write_pass": nw, "write_size_kib": w, "write_bytes": None if w is None else w * 1024}
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    print("wrote", sorted(os.listdir(dst)))


if __name__ == "__main__":
    main(*sys.argv[1:])
