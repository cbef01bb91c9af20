mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tbd.py tests/test_gpu_tbd_e2e.py > gpurun_out/t_pd.log 2>&1; tail -2 gpurun_out/t_pd.log
grep -q " passed" gpurun_out/t_pd.log && ! grep -q "failed" gpurun_out/t_pd.log || exit 1
L=opencv_amd/lib/libtbdk.so
bash tools/ab.sh 4 pd=$L old=$L,--ctx-option=tbd_post_direct=0 || exit 1
