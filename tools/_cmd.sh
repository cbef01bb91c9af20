set -e
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_farneback.py > gpurun_out/t39.log 2>&1 || { tail -30 gpurun_out/t39.log; exit 1; }
tail -1 gpurun_out/t39.log
for i in 1 2; do
for v in base cur; do
  lib=$R/tools/bin/libtbdk_base.so; [ $v = cur ] && lib=$R/opencv_amd/lib/libtbdk.so
  TBDK_LIB=$lib timeout -k 10 120 python tools/bench_farneback.py --pairs 20 > gpurun_out/fb_$v.json 2>/dev/null
  TBDK_LIB=$lib timeout -k 10 120 python tools/bench_farneback.py --pairs 20 --flags 256 > gpurun_out/fg_$v.json 2>/dev/null
  python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['kernels']['fb_iter']['avg_us'])" gpurun_out/fb_$v.json gpurun_out/fg_$v.json
done
done
