set -o pipefail
B="python bench.py --steps 1500 --no-cpu-baseline --no-step-api --no-farneback --no-hog --no-f16"
for i in 1 2 3; do
for p in 0 1; do
TBDK_LA_PRIO=$p timeout -k 10 200 $B > gpurun_out/ab_la${p}_$i.json 2>/dev/null || exit 1
done
done
