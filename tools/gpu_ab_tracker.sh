set -e
for i in 1 2; do tools/bin/bench_tracker_old 128 r 20; tools/bin/bench_tracker_new 128 r 20; done > gpurun_out/trk.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_tbd.py tests/test_gpu_tbd_e2e.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_tbd.log 2>&1
timeout -k 10 700 bash tools/ab.sh 3 new=opencv_amd/lib/libtbdk.so old=tools/bin/libtbdk_old.so > gpurun_out/ab1.txt 2>&1
for i in 1 2 3; do for v in new=opencv_amd/lib/libtbdk.so old=tools/bin/libtbdk_old.so; do TBDK_LIB=${v#*=} timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/drv_${v%%=*}_$i.json 2>/dev/null; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['per_frame']['host_tracker_us'], d['per_frame']['host_step_us'])" gpurun_out/drv_${v%%=*}_$i.json ${v%%=*}; done; done > gpurun_out/drv.txt 2>&1
