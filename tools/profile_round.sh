#!/usr/bin/env bash
# profile_round.sh <round tag, e.g. r02> — the committed profiles of a round:
#   profiles/<tag>_kernel_stats.csv : rocprofv3 --kernel-trace --stats of the default bench.py
#   profiles/<tag>_bench.json       : that run's bench line
#   profiles/<tag>_pmc.json         : FETCH_SIZE / WRITE_SIZE, separate --pmc passes (bench.py --steps 60, reduced secondaries)
#
# Run on the GPU box (gpurun); only gpurun_out/ comes back, so then run
#   tools/profile_round.sh --collect <tag>
# here to copy the summaries into profiles/.
set -euo pipefail
if [ "${1:-}" = "--collect" ]; then
    tag=$2; out=gpurun_out/prof_$tag
    cp "$out"/stats/kt_kernel_stats.csv "profiles/${tag}_kernel_stats.csv"
    tail -n 1 "$out/bench.json" > "profiles/${tag}_bench.json"
    cp "$out/pmc.json" "profiles/${tag}_pmc.json"
    exit 0
fi
tag=$1
root=$(pwd); out=$root/gpurun_out/prof_$tag; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o kt \
    -- python3 "$root/bench.py" > "$out/bench.json" 2> "$out/bench.err"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/$c" -o pmc \
        -- python3 "$root/bench.py" --steps 60 --sequence-frames 100 --no-cpu-baseline --no-step-api --repeats 0 \
        --no-h2d --no-kitti --fb-pairs 3 --f16-pairs 3 --hog-frames 10 > "$out/$c.json" 2> "$out/$c.err"
done
python3 "$root/tools/pmc_json.py" "$out/FETCH_SIZE/pmc_counter_collection.csv" "$out/WRITE_SIZE/pmc_counter_collection.csv" \
    "$out/pmc.json" \
    "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (kernel trace only), bench.py --steps 60 --sequence-frames 100 --no-cpu-baseline --no-step-api --repeats 0 --no-h2d --no-kitti --fb-pairs 3 --f16-pairs 3 --hog-frames 10; per-launch means; FETCH_SIZE/WRITE_SIZE are KiB; fetch_bytes = 2 x FETCH_SIZE (the guide's gfx950 correction for wide 16-B-per-lane reads, MI355X_MICROARCH.md HBM section), fetch_size_kib is the raw count that bench.py's roofline traffic uses (its kernels load <= 4 B per lane); Infinity-Cache hits are included in these memory-side counters."
