#!/usr/bin/env bash
# pmc_pyr_fp.sh <outdir> [probe filter, default 3840x2160:float16:uint8 | u8] -- counters of the
# role-split fp pyramid build (tools/probe_pyr_fp.py, one configuration) or, with "u8", of the
# u8 two-role levels-only build (tools/probe_pyr.py "two-role r1": 1080p, KITTI, 4K): one
# rocprofv3 --pmc pass per counter group (<= 8 SQ + GRBM, then FETCH_SIZE, then WRITE_SIZE),
# kernel trace only; summary per (kernel, grid size) in <outdir>/summary.json.  GPU box.
set -euo pipefail
root=$(pwd); out=$root/$1; cfg=${2:-3840x2160:float16:uint8}
mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    if [ "$cfg" = u8 ]; then
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o pmc \
            -- python3 "$root/tools/probe_pyr.py" "two-role r1" > "$out/p$i.log" 2>&1
    else
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o pmc \
            -- python3 "$root/tools/probe_pyr_fp.py" "$cfg" > "$out/p$i.log" 2>&1
    fi
done
python3 - "$out" <<'PY'
import collections, csv, glob, json, os, sys
out = sys.argv[1]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(p)):
        if "pyr" not in r["Kernel_Name"] and "scharr" not in r["Kernel_Name"] and "pad_copy" not in r["Kernel_Name"]:
            continue
        key = f'{r["Kernel_Name"][:70]} grid={r.get("Grid_Size", r.get("Grid_Size_X", "?"))}'
        d[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, c in d.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    e = {"launches": max(len(v) for v in c.values()), **{n: round(x, 1) for n, x in m.items()}}
    if "GRBM_GUI_ACTIVE" in m:
        clk = m["GRBM_GUI_ACTIVE"] / 8
        e["duration_us_at_2400MHz"] = round(clk / 2400, 2)
        if "SQ_WAVE_CYCLES" in m:
            e["waves_per_simd"] = round(4 * m["SQ_WAVE_CYCLES"] / clk / 1024, 2)
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU"):
            if n in m:
                e[n.lower() + "_share"] = round(m[n] / m["SQ_WAVE_CYCLES"], 3)
    if "FETCH_SIZE" in m:
        e["fetch_mb"] = round(m["FETCH_SIZE"] * 1024 / 1e6, 2)
    if "WRITE_SIZE" in m:
        e["write_mb"] = round(m["WRITE_SIZE"] * 1024 / 1e6, 2)
    res[k] = e
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k, e in sorted(res.items()):
    print(k, json.dumps(e))
PY
