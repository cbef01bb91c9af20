#!/usr/bin/env python3
"""Per-frame GPU timeline of a `rocprofv3 --kernel-trace --memory-copy-trace
--output-format csv` run of bench.py: busy fraction (union of kernel and copy
intervals), per-kernel mean duration, and an event listing of a few frames
(times relative to each frame's first pyramid kernel).

usage: tools/timeline.py <dir with *_kernel_trace.csv> [--frames 3] [--skip 40]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("tbdk::", "")
    return n[:28]


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                       "q%s" % r["Queue_Id"]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H" if "DEVICE_TO_HOST" in r["Direction"] else "copy"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, "dma"))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--skip", type=int, default=40)
    ap.add_argument("--first", default="pad_copy_kernel")
    a = ap.parse_args()
    ev = [e for e in load(a.dir) if "synth" not in e[2]]
    starts = [i for i, e in enumerate(ev) if e[2].startswith(a.first)]
    if len(starts) < a.skip + 2:
        a.skip = max(0, len(starts) // 3)
    lo, hi = ev[starts[a.skip]][0], ev[starts[-2]][0]
    nfr = len(starts) - 2 - a.skip
    win = [e for e in ev if lo <= e[0] < hi]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += min(cur_e, hi) - cur_s
    per = defaultdict(list)
    for s, e, n, _ in win:
        per[n].append(e - s)
    print(f"frames {nfr}: wall {(hi - lo) / nfr / 1e3:.1f} us/frame, GPU busy {busy / nfr / 1e3:.1f} us/frame "
          f"({100.0 * busy / (hi - lo):.0f}%)")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:30s} {len(v) / nfr:5.2f}/frame  mean {sum(v) / len(v) / 1e3:7.1f} us  "
              f"total {sum(v) / nfr / 1e3:7.1f} us/frame")
    for k in range(a.frames):
        i0, i1 = starts[a.skip + k], starts[a.skip + k + 1]
        t0 = ev[i0][0]
        print(f"-- frame (+{k})")
        for s, e, n, q in ev:
            if ev[i0][0] - 150_000 <= s < ev[i1][0]:
                print(f"   {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  {q:4s} {n}")


if __name__ == "__main__":
    main()
