mkdir -p gpurun_out/tl3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tbd.py > gpurun_out/t_tbd.log 2>&1; tail -3 gpurun_out/t_tbd.log
root=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $root/gpurun_out/tl3 -o kt -- python3 $root/bench.py --no-secondary --no-cpu-baseline --ctx-option tbd_early_la=3 > $root/gpurun_out/tl3/bench.json 2> $root/gpurun_out/tl3/bench.err || exit 1
cd $root
python3 tools/timeline.py gpurun_out/tl3 --first pyr_build_kernel --skip 100 --frames 6 > gpurun_out/tl3/timeline.txt
head -40 gpurun_out/tl3/timeline.txt
bash tools/ab.sh 3 la1=opencv_amd/lib/libtbdk.so la3=opencv_amd/lib/libtbdk.so,--ctx-option=tbd_early_la=3
