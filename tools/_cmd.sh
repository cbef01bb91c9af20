set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_hog.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_hog.log 2>&1 || exit 1
