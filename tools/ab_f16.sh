set -e
for i in 1 2 3; do for v in base:opencv_amd/lib/libtbdk_base.so new:opencv_amd/lib/libtbdk.so; do n=${v%%:*}; l=${v#*:}
TBDK_LIB=$l timeout -k 10 200 python bench.py --steps 20 --warmup 5 --sequence-frames 25 --no-cpu-baseline --no-step-api --repeats 0 --no-h2d --no-kitti --no-farneback --no-hog --no-copy-peak --f16-pairs 20 > gpurun_out/ab16_${n}_$i.json 2> gpurun_out/ab16_${n}_$i.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['lk_f16']; print(sys.argv[2], d['value'], d['kernels']['lk_sparse']['avg_us'], d['roofline']['frac'])" gpurun_out/ab16_${n}_$i.json $n
done; done
