#!/usr/bin/env bash
# r06_fb_lds.sh — GPU box: LDS counters of fb_iter per level (grid size), the
# default build against the half-wave horizontal pass (TBDK_FB_HX=1, round 4's
# rejected build): one --pmc pass of 8 SQ counters per build over a short 4K
# Farneback probe (tools/bench_farneback.py, box blur), kernel trace only.
set -euo pipefail
root=$(pwd); cd /tmp; export TMPDIR=/tmp
ctr="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"
for v in ${FB_LDS_VARIANTS:-default=$root/opencv_amd/lib/libtbdk.so hx=$root/opencv_amd/lib/libtbdk_fbhx.so}; do
    name=${v%%=*}; lib=${v#*=}; out=$root/gpurun_out/fblds_$name; mkdir -p "$out"
    TBDK_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$out" -o pmc \
        -- python3 "$root/tools/bench_farneback.py" --pairs 2 --warmup 1 --flags 0 > "$out/bench.json" 2> "$out/err.txt"
    f=$(find "$out" -name 'pmc_counter_collection.csv' | head -1)
    python3 "$root/tools/pmc_by_grid.py" "$f" fb_iter > "$out/by_grid.txt"
done
