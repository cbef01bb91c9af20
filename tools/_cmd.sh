mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gftt.py tests/test_gpu_tbd.py > gpurun_out/t_gf.log 2>&1; tail -2 gpurun_out/t_gf.log
grep -q " passed" gpurun_out/t_gf.log && ! grep -q "failed" gpurun_out/t_gf.log || exit 1
L=opencv_amd/lib/libtbdk.so
bash tools/ab.sh 3 gin=$L gmem=$L,--ctx-option=gftt_inline=0 || exit 1
