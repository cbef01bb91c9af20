set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_klt.py tests/test_gpu_tbd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_klt.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_klt.py > gpurun_out/probe_d.log 2>&1 || exit 1
root=$PWD; mkdir -p gpurun_out/trace; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $root/gpurun_out/trace -o kt -- python3 $root/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-step-api --no-farneback --no-hog > $root/gpurun_out/bench_tr.json 2>/dev/null || exit 1
