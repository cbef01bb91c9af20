#!/usr/bin/env python3
"""Critical-chain gaps of the TBD loop from a rocprofv3 --kernel-trace csv of
bench.py: per frame (one fit kernel each), the fit's start after the end of
the PyrLK launch before it on the fit's queue, the next critical PyrLK's start
after the fit's end, and the critical PyrLK's duration; medians over the
middle frames, plus one frame's kernel listing.
usage: tools/chain_gaps.py <kernel_trace.csv> [frame to list]"""
import csv
import re
import statistics as st
import sys


def main(path, show=None):
    ev = []
    for r in csv.DictReader(open(path)):
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("tbdk::", "").replace("void ", "")[:30]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
    ev.sort()
    fits = [i for i, e in enumerate(ev) if "fit" in e[2]]
    fq = ev[fits[len(fits) // 2]][3]
    lo, hi = len(fits) // 5, 4 * len(fits) // 5
    g_fit, g_lk, d_lk, frame = [], [], [], []
    for a, b in zip(fits[lo:hi], fits[lo + 1:hi + 1]):
        fs, fe = ev[a][0], ev[a][1]
        prev = [e for e in ev[max(0, a - 12):a] if e[3] == fq and "lk_multi" in e[2]]
        if prev:
            g_fit.append((fs - max(e[1] for e in prev)) / 1e3)
        crit = [e for e in ev[a + 1:b] if e[3] == fq and "lk_multi" in e[2]]
        if crit:
            g_lk.append((crit[0][0] - fe) / 1e3)
            d_lk.append((crit[0][1] - crit[0][0]) / 1e3)
        frame.append((ev[b][1] - fe) / 1e3)
    q = lambda v: "median %.1f  p10 %.1f  p90 %.1f" % (st.median(v), sorted(v)[len(v) // 10], sorted(v)[9 * len(v) // 10])
    print("frames", len(frame), "fit end -> fit end:", q(frame))
    print("PyrLK end -> fit start (same queue):", q(g_fit))
    print("fit end -> critical PyrLK start:", q(g_lk))
    print("critical PyrLK duration:", q(d_lk))
    if show is not None:
        a = fits[int(show)]
        b = fits[int(show) + 2]
        t0 = ev[a][1]
        for s, e, n, qq in ev:
            if ev[a][0] - 100000 <= s < ev[b][1]:
                print("%8.1f %8.1f %7.1f q%s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, qq, n))


if __name__ == "__main__":
    main(*sys.argv[1:])
