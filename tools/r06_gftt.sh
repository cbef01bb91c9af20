#!/usr/bin/env bash
# r06_gftt.sh — GPU box: GFTT compact-candidate mode (ctx option gftt_compact):
# parity tests, loop A/B against the dense eigenvalue plane, and loop-only
# FETCH_SIZE / WRITE_SIZE passes (kernel trace only) for the new default.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gftt.py tests/test_gpu_tbd.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/t_gftt.log 2>&1
bash tools/ab.sh 3 compact=opencv_amd/lib/libtbdk.so dense=opencv_amd/lib/libtbdk.so,--ctx-option,gftt_compact=0 \
    > gpurun_out/ab3.txt 2>&1
root=$(pwd); out=$root/gpurun_out/pmc_r06a; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/loop_$c" -o pmc \
        -- python3 "$root/bench.py" --no-secondary --no-cpu-baseline > "$out/loop_$c.json" 2> "$out/loop_$c.err"
done
python3 "$root/tools/pmc_json.py" "$out/loop_FETCH_SIZE/pmc_counter_collection.csv" \
    "$out/loop_WRITE_SIZE/pmc_counter_collection.csv" "$out/pmc_loop.json" "r06 GFTT compact, loop only"
