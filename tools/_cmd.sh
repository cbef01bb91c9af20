set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_farneback.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_fb.log 2>&1 || exit 1
for f in 0 256; do
timeout -k 10 200 python tools/bench_farneback.py --pairs 10 --flags $f > gpurun_out/fbn_$f.json 2>/dev/null || exit 1
TBDK_LIB=opencv_amd/lib/var_head.so timeout -k 10 200 python tools/bench_farneback.py --pairs 10 --flags $f > gpurun_out/fbh_$f.json 2>/dev/null || exit 1
done
