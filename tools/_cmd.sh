mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tbd.py tests/test_gpu_tbd_e2e.py > gpurun_out/t_wg.log 2>&1; tail -2 gpurun_out/t_wg.log
grep -q " passed" gpurun_out/t_wg.log && ! grep -q "failed" gpurun_out/t_wg.log || exit 1
L=opencv_amd/lib/libtbdk.so
bash tools/ab.sh 3 wg=$L wave=$L,--ctx-option=tbd_fit_wgpub=0 || exit 1
bash tools/ab.sh 2 dwg=$L,--steps=20,--warmup=5 dwave=$L,--ctx-option=tbd_fit_wgpub=0,--steps=20,--warmup=5 || exit 1
