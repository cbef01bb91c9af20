#!/usr/bin/env bash
# ab_env.sh N name=VAR=value ... -- N alternating rounds of the loop-only bench (480 frames and the
# driver's shape) per environment variant ("base=" runs with the environment as it is)
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        name=${spec%%=*}; kv=${spec#*=}
        for shape in long drv; do
            flags="--no-secondary --no-cpu-baseline"
            [ "$shape" = drv ] && flags="$flags --steps 20 --warmup 5"
            if [ -n "$kv" ]; then
                env "$kv" timeout -k 10 120 python bench.py $flags > "gpurun_out/env_${name}_${shape}_${i}.json" 2>/dev/null
            else
                timeout -k 10 120 python bench.py $flags > "gpurun_out/env_${name}_${shape}_${i}.json" 2>/dev/null
            fi
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'])" \
                "gpurun_out/env_${name}_${shape}_${i}.json" "$name" "$shape"
        done
    done
done
