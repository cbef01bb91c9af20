#!/usr/bin/env bash
# ab_fb.sh N name=lib ... -- A/B builds of libtbdk on the 4K Farneback probe:
# N alternating rounds of tools/bench_farneback.py per variant, box blur
# (flags 0) and Gaussian (flags 256); run on the GPU box.
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        name=${spec%%=*}; lib=${spec#*=}
        for fl in 0 256; do
            TBDK_LIB=$lib timeout -k 10 120 python tools/bench_farneback.py --pairs 10 --flags $fl \
                > "gpurun_out/abfb_${name}_${fl}_${i}.json" 2> "gpurun_out/abfb_${name}_${fl}_${i}.err"
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value'],1), round(d['kernels']['fb_iter']['avg_us'],2), round(d['roofline_fb_iter']['frac'],4))" \
                "gpurun_out/abfb_${name}_${fl}_${i}.json" "$name" "$fl"
        done
    done
done
