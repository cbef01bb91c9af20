set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_klt.py tests/test_gpu_tbd.py tests/test_gpu_dense_lk.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_klt.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_lk_scale.py > gpurun_out/probe_scale_new.txt 2>&1 || exit 1
TBDK_LIB=opencv_amd/lib/var_head.so timeout -k 10 120 python tools/probe_lk_scale.py > gpurun_out/probe_scale_head.txt 2>&1 || exit 1
B="python bench.py --steps 1500 --no-cpu-baseline --no-step-api --no-farneback --no-hog --no-f16"
for i in 1 2 3; do
timeout -k 10 200 $B > gpurun_out/ab_new_$i.json 2>/dev/null || exit 1
TBDK_LIB=opencv_amd/lib/var_head.so timeout -k 10 200 $B > gpurun_out/ab_head_$i.json 2>/dev/null || exit 1
done
