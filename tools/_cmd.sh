set -o pipefail
B="python bench.py --steps 1500 --no-cpu-baseline --no-step-api --no-farneback --no-hog --no-f16"
for i in 1 2 3; do
timeout -k 10 200 $B > gpurun_out/ab_hs0_$i.json 2>/dev/null || exit 1
TBDK_HI_STREAM=1 timeout -k 10 200 $B > gpurun_out/ab_hs1_$i.json 2>gpurun_out/ab_hs1.err || exit 1
done
