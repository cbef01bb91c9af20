set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in flag event; do
  fl=1; [ $v = event ] && fl=0
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gt_$v -o kt -- python3 $R/bench.py --no-secondary --no-cpu-baseline --repeats 0 --no-h2d --no-kitti --no-step-api --ctx-option tbd_fit_flag=$fl > $R/gpurun_out/gt_$v.json 2> $R/gpurun_out/gt_$v.err
  python3 $R/tools/gaps.py $R/gpurun_out/gt_$v/kt_kernel_trace.csv
done
