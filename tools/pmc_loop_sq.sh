#!/usr/bin/env bash
# pmc_loop_sq.sh <tag> — SQ (+ GRBM) counters of the TBD loop's kernels as they
# run inside the loop (bench.py's contract leg only, 100 timed frames), one
# rocprofv3 --pmc pass per counter group (<= 8 SQ, <= 2 GRBM each), kernel trace
# only.  Then tools/pmc_sq_json.py merges the passes into gpurun_out/sq_<tag>/sq.json
# (per-kernel means and the derived issue / occupancy figures).
set -euo pipefail
tag=$1
root=$(pwd); out=$root/gpurun_out/sq_$tag; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_LEVEL_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o pmc \
        -- python3 "$root/bench.py" --steps 100 --sequence-frames 130 --no-secondary --no-cpu-baseline \
        > "$out/p$i.json" 2> "$out/p$i.err" || echo "pass $i failed (rc $?)"
done
python3 "$root/tools/pmc_sq_json.py" "$out/sq.json" "$out"/p*/pmc_counter_collection.csv
