#!/usr/bin/env bash
# pmc_quick.sh <outdir> <counter> [bench args...] — one --pmc pass over a short bench run
set -euo pipefail
root=$(pwd); out=$root/$1; ctr=$2; shift 2
mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv -d "$out" -o pmc \
    -- python3 "$root/bench.py" --steps 40 --no-cpu-baseline "$@" > "$out/bench.json" 2> "$out/err.txt"
python3 - "$out/pmc_counter_collection.csv" <<'PY'
import csv, collections, sys
d = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    d[row["Kernel_Name"][:60]].append(float(row["Counter_Value"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:60s} n={len(v):4d} mean={sum(v)/len(v):12.1f}")
PY
