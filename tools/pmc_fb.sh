#!/usr/bin/env bash
# pmc_fb.sh <outdir> <counters> [bench_farneback args...] — one --pmc pass over a
# short Farneback probe run; prints per-kernel mean counter values.
set -euo pipefail
root=$(pwd); out=$root/$1; ctr=$2; shift 2
mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$out" -o pmc \
    -- python3 "$root/tools/bench_farneback.py" --pairs 2 --warmup 1 "$@" > "$out/bench.json" 2> "$out/err.txt"
python3 - "$out" <<'PY'
import csv, collections, glob, os, sys
f = glob.glob(os.path.join(sys.argv[1], "**", "pmc_counter_collection.csv"), recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f)):
    d[row["Kernel_Name"][:70]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(d.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} n={len(v):4d} mean={sum(v)/len(v):16.1f} sum={sum(v):18.1f}")
PY
