set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_hog.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_hog.log 2>&1 || exit 1
B="python bench.py --steps 20 --no-cpu-baseline --no-step-api --no-farneback --no-f16"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/hog_new_$i.json 2>/dev/null || exit 1
TBDK_LIB=opencv_amd/lib/var_head.so timeout -k 10 300 $B > gpurun_out/hog_head_$i.json 2>/dev/null || exit 1
done
