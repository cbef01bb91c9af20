set -o pipefail
B="python bench.py --steps 1500 --no-cpu-baseline --no-step-api --no-farneback --no-hog --no-f16"
for i in 1 2 3 4; do
timeout -k 10 200 $B > gpurun_out/ab_new_$i.json 2>/dev/null || exit 1
TBDK_LIB=opencv_amd/lib/var_head.so timeout -k 10 200 $B > gpurun_out/ab_head_$i.json 2>/dev/null || exit 1
done
