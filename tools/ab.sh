#!/usr/bin/env bash
# ab.sh N name=lib[,bench flags] ... -- A/B builds / options of libtbdk on the
# frame loop: N alternating rounds of `bench.py --no-secondary --no-cpu-baseline`
# per variant (TBDK_LIB = lib; extra bench flags after commas, e.g.
# "planes=opencv_amd/lib/libtbdk.so,--pyr-derivs"), each line to
# gpurun_out/ab_<name>_<round>.json; run on the GPU box.
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; flags=""
        [ "$rest" != "$lib" ] && flags=${rest#*,} && flags=${flags//,/ }
        TBDK_LIB=$lib timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline $flags \
            > "gpurun_out/ab_${name}_${i}.json" 2> "gpurun_out/ab_${name}_${i}.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_us_sampled'])" \
            "gpurun_out/ab_${name}_${i}.json" "$name"
    done
done
