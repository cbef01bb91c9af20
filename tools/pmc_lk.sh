#!/usr/bin/env bash
# pmc_lk.sh <outdir> — SQ counter passes over tools/probe_klt.py (every LK kernel
# variant on the same 1080p x 32k-point pair); one rocprofv3 --pmc run per pass.
set -euo pipefail
root=$(pwd); out=$root/$1; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o pmc \
        -- python3 "$root/tools/probe_klt.py" > "$out/$name.log" 2>&1
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass b SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
python3 "$root/tools/pmc_summary.py" "$out"/a/pmc_counter_collection.csv "$out"/b/pmc_counter_collection.csv > "$out/summary.txt"
