mkdir -p gpurun_out/tl
root=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $root/gpurun_out/tl -o kt -- python3 $root/bench.py --no-secondary --no-cpu-baseline > $root/gpurun_out/tl/bench.json 2> $root/gpurun_out/tl/bench.err || exit 1
cd $root
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py gpurun_out/tl --first pyr_build_kernel --skip 100 --frames 4 > gpurun_out/tl/timeline.txt
python3 tools/gaps.py $f > gpurun_out/tl/gaps.txt
head -30 gpurun_out/tl/timeline.txt
