#!/usr/bin/env bash
# profile_round.sh <round tag, e.g. r02> — the committed profiles of a round:
#   profiles/<tag>_kernel_stats.csv : rocprofv3 --kernel-trace --stats of the default bench.py
#   profiles/<tag>_bench.json       : that run's bench line
#   profiles/<tag>_ktrace_grid.json : that run's kernel-trace durations per (kernel, grid size) (tools/ktrace_by_grid.py)
#   profiles/<tag>_kernel_stats_loop.csv : --kernel-trace --stats of bench.py --no-secondary (configs[2]'s loop only:
#                                     the roofline's frac_kernel_trace_loop)
#   profiles/<tag>_pmc_loop.json    : FETCH_SIZE / WRITE_SIZE of the contract's legs only (bench.py --no-secondary:
#                                     the 1080p x 128 loop), separate --pmc passes -- the loop kernels' traffic fields
#   profiles/<tag>_pmc.json         : FETCH_SIZE / WRITE_SIZE, separate --pmc passes (bench.py --steps 60, reduced
#                                     secondaries) -- the secondaries' kernels (fb_iter)
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
    cp "$out/pmc_loop.json" "profiles/${tag}_pmc_loop.json"
    cp "$out/ktrace_grid.json" "profiles/${tag}_ktrace_grid.json"
    cp "$out"/stats_loop/kt_kernel_stats.csv "profiles/${tag}_kernel_stats_loop.csv"
    exit 0
fi
tag=$1
root=$(pwd); out=$root/gpurun_out/prof_$tag; mkdir -p "$out"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o kt \
    -- python3 "$root/bench.py" > "$out/bench.json" 2> "$out/bench.err"
python3 "$root/tools/ktrace_by_grid.py" "$out/stats/kt_kernel_trace.csv" "$out/ktrace_grid.json" \
    "rocprofv3 --kernel-trace --stats of the default bench.py (this round's kernel_stats run): per (kernel, grid) GPU durations" \
    > /dev/null
# the contract's loop alone (bench.py --no-secondary): kernel-trace durations of configs[2]'s launches only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_loop" -o kt \
    -- python3 "$root/bench.py" --no-secondary --no-cpu-baseline > "$out/bench_loop.json" 2> "$out/bench_loop.err"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/loop_$c" -o pmc \
        -- python3 "$root/bench.py" --no-secondary --no-cpu-baseline > "$out/loop_$c.json" 2> "$out/loop_$c.err"
done
python3 "$root/tools/pmc_json.py" "$out/loop_FETCH_SIZE/pmc_counter_collection.csv" \
    "$out/loop_WRITE_SIZE/pmc_counter_collection.csv" "$out/pmc_loop.json" \
    "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (kernel trace only) over bench.py --no-secondary --no-cpu-baseline: only the contract's 1080p x 128 loop (warm-up and timed frames) runs, so every launch counted is configs[2]'s; per-launch means; FETCH_SIZE/WRITE_SIZE are KiB; fetch_bytes = 2 x FETCH_SIZE (the guide's wide-read correction), fetch_size_kib is the raw count bench.py's loop traffic fields use (4 B per lane loads)"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/$c" -o pmc \
        -- python3 "$root/bench.py" --steps 60 --sequence-frames 100 --no-cpu-baseline --no-step-api --repeats 0 \
        --no-h2d --no-kitti --fb-pairs 3 --f16-pairs 3 --hog-frames 10 > "$out/$c.json" 2> "$out/$c.err"
done
python3 "$root/tools/pmc_json.py" "$out/FETCH_SIZE/pmc_counter_collection.csv" "$out/WRITE_SIZE/pmc_counter_collection.csv" \
    "$out/pmc.json" \
    "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (kernel trace only), bench.py --steps 60 --sequence-frames 100 --no-cpu-baseline --no-step-api --repeats 0 --no-h2d --no-kitti --fb-pairs 3 --f16-pairs 3 --hog-frames 10; per-launch means; FETCH_SIZE/WRITE_SIZE are KiB; fetch_bytes = 2 x FETCH_SIZE (the guide's gfx950 correction for wide 16-B-per-lane reads, MI355X_MICROARCH.md HBM section), fetch_size_kib is the raw count that bench.py's roofline traffic uses (its kernels load <= 4 B per lane); Infinity-Cache hits are included in these memory-side counters."
