#!/usr/bin/env bash
# pmc_gftt.sh <outdir> [nroi] — kernel stats and SQ counter passes over
# tools/probe_gftt.py (GFTT alone on the bench frame's boxes); one rocprofv3 run per pass.
set -euo pipefail
root=$(pwd); out=$root/$1; nroi=${2:-128}; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o k \
    -- python3 "$root/tools/probe_gftt.py" 50 "$nroi" > "$out/stats.log" 2>&1
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o pmc \
        -- python3 "$root/tools/probe_gftt.py" 20 "$nroi" > "$out/$name.log" 2>&1
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass b SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
pass c SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH
python3 "$root/tools/pmc_summary.py" "$out"/a/pmc_counter_collection.csv "$out"/b/pmc_counter_collection.csv "$out"/c/pmc_counter_collection.csv > "$out/summary.txt"
