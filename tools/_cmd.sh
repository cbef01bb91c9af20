mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1; tail -2 gpurun_out/gpu_full.log
grep -q " passed" gpurun_out/gpu_full.log && ! grep -q "failed" gpurun_out/gpu_full.log || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
grep -q __SMOKE_OK__ gpurun_out/smoke.log || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
for i in 1 2; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_$i.json 2> gpurun_out/bench_drv_$i.err || exit 1; done
bash tools/profile_round.sh r05 > gpurun_out/prof_r05.log 2>&1 || { tail -5 gpurun_out/prof_r05.log; exit 1; }
