set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest_final.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/drv_$i.json 2> gpurun_out/drv_$i.err; done
