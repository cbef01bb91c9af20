set -e
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_tbd.py tests/test_gpu_tbd_e2e.py > gpurun_out/t37.log 2>&1 || { tail -30 gpurun_out/t37.log; exit 1; }
tail -1 gpurun_out/t37.log
bash tools/ab.sh 3 pre=$PWD/opencv_amd/lib/libtbdk.so nopre=$PWD/opencv_amd/lib/libtbdk.so,--ctx-option=tbd_la_prewait=0
