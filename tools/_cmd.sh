mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tbd.py tests/test_gpu_hog.py > gpurun_out/t_tbd.log 2>&1; tail -2 gpurun_out/t_tbd.log
grep -q " passed" gpurun_out/t_tbd.log && ! grep -q "failed" gpurun_out/t_tbd.log || exit 1
timeout -k 10 800 python -u bench.py --no-cpu-baseline > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit 1
