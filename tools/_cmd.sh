set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_f16.py tests/test_gpu_klt.py tests/test_gpu_dense_lk.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_f16.log 2>&1 || exit 1
