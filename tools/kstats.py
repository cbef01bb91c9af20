#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 results database (rocpd sqlite)."""
import sqlite3
import sys


def main(path, out=None):
    c = sqlite3.connect(path)
    q = ("select name, count(*), avg(end-start)/1000.0, min(end-start)/1000.0, max(end-start)/1000.0, "
         "sum(end-start)/1e6 from kernels group by name order by sum(end-start) desc")
    lines = ["name,calls,avg_us,min_us,max_us,total_ms"]
    for n, k, a, mn, mx, t in c.execute(q):
        lines.append(f'"{n}",{k},{a:.2f},{mn:.2f},{mx:.2f},{t:.3f}')
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
