#!/usr/bin/env bash
# profile_round.sh <tag> — run on the GPU box (via gpurun) from the repo root.
# 1. kernel trace + stats of the default bench command (the judged run shape);
# 2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (they cannot share one
#    pass on gfx950), each with kernel trace only, on a shorter bench run.
# Outputs land in gpurun_out/prof_<tag>/; tools/summarize_profiles.py turns
# them into the committed profiles/<tag>_*.csv / .json files.
set -euo pipefail
tag=${1:-r01}
root=$(pwd)
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o bench \
    -- python3 "$root/bench.py" > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/fetch" -o bench \
    -- python3 "$root/bench.py" --steps 60 --no-cpu-baseline > "$out/bench_fetch.json" 2> "$out/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out/write" -o bench \
    -- python3 "$root/bench.py" --steps 60 --no-cpu-baseline > "$out/bench_write.json" 2> "$out/write.err"
ls -R "$out" | head -50
