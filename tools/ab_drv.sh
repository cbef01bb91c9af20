#!/usr/bin/env bash
# ab_drv.sh N name=lib[,flags] ... -- the driver's shape (bench.py --steps 20 --warmup 5, loop only) per
# variant, N alternating rounds; prints name, value, sampled PyrLK us (GPU box)
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; flags=""
        [ "$rest" != "$lib" ] && flags=${rest#*,} && flags=${flags//,/ }
        TBDK_LIB=$lib timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline $flags \
            > "gpurun_out/drv_${name}_${i}.json" 2> "gpurun_out/drv_${name}_${i}.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_us_sampled'])" \
            "gpurun_out/drv_${name}_${i}.json" "$name"
    done
done
