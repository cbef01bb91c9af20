set -o pipefail
timeout -k 10 120 python tools/probe_klt.py > gpurun_out/probe_m3.log 2>&1 || exit 1
TBDK_LIB=$PWD/opencv_amd/lib/alt/libtbdk_w4.so timeout -k 10 120 python tools/probe_klt.py > gpurun_out/probe_m3w4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 240 --no-cpu-baseline --no-step-api --no-farneback --no-hog > gpurun_out/bench_m3.json 2>/dev/null || exit 1
TBDK_LIB=$PWD/opencv_amd/lib/alt/libtbdk_w4.so timeout -k 10 200 python bench.py --steps 240 --no-cpu-baseline --no-step-api --no-farneback --no-hog > gpurun_out/bench_m3w4.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 240 --no-cpu-baseline --no-step-api --no-farneback --no-hog --lk-impl 1 > gpurun_out/bench_m3s.json 2>/dev/null || exit 1
