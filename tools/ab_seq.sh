#!/usr/bin/env bash
# ab_seq.sh N name=lib[,bench flags] ... -- A/B of the bench's whole-sequence leg (500 frames after
# 20 warm-up, fresh loop per run, median of 5) and its timed region: N alternating rounds per
# variant, every other secondary off; lines to gpurun_out/abseq_<name>_<round>.json.  GPU box.
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; flags=""
        [ "$rest" != "$lib" ] && flags=${rest#*,}
        TBDK_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-step-api --no-h2d --no-kitti \
            --no-bounds-frame --no-pyr4k --no-farneback --no-f16 --no-copy-peak --no-hog $flags \
            > "gpurun_out/abseq_${name}_${i}.json" 2> "gpurun_out/abseq_${name}_${i}.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['sequence']['median_fps'], d['sequence'].get('runs_fps'))" \
            "gpurun_out/abseq_${name}_${i}.json" "$name"
    done
done
