"""Idle gaps of the device in a rocprofv3 kernel trace (--kernel-trace csv):
the union of kernel intervals over the timed frames of a bench run, and the
gaps between consecutive busy intervals classified by the kernels on either
side.  Usage: python tools/gaps.py <kernel_trace.csv> [first_lk last_lk]"""
import collections
import csv
import sys


def main(path, a=None, b=None):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("::")[-1][:26])
                for r in csv.DictReader(open(path)))
    lk = [e for e in ev if "lk_multi" in e[2]]
    a = int(a) if a else len(lk) // 4
    b = int(b) if b else 3 * len(lk) // 4
    t0, t1 = lk[a][0], lk[b][0]
    sel = [e for e in ev if e[0] >= t0 and e[1] <= t1]
    gaps, gsum = collections.Counter(), collections.Counter()
    busy, cs, ce, prev = 0, sel[0][0], sel[0][1], sel[0][2]
    for s, e, n in sel[1:]:
        if s > ce:
            busy += ce - cs
            if s - ce < 2_000_000:  # run boundaries excluded
                gaps[(prev, n)] += 1
                gsum[(prev, n)] += s - ce
            cs, ce, prev = s, e, n
        elif e > ce:
            ce, prev = e, n
    busy += ce - cs
    print(f"window {(t1 - t0) / 1e3:.0f} us, busy {busy / 1e3:.0f} us ({busy / (t1 - t0):.3f}), "
          f"lk launches {b - a}, gaps {sum(gsum.values()) / 1e3:.0f} us")
    for k, v in gsum.most_common(8):
        print(f"  {k[0]:>26s} -> {k[1]:<26s} n={gaps[k]:5d} total {v / 1e3:8.1f} us  mean {v / gaps[k] / 1e3:6.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
