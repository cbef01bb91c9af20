#!/usr/bin/env bash
# ab_pyr.sh N name=lib ... -- N alternating rounds of tools/probe_pyr_build.py per library (GPU box)
set -euo pipefail
n=$1; shift
for i in $(seq 1 "$n"); do
    for spec in "$@"; do
        echo "${spec%%=*} $(TBDK_LIB=${spec#*=} timeout -k 10 120 python tools/probe_pyr_build.py)"
    done
done
