set -e
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_tbd.py tests/test_gpu_tbd_e2e.py tests/test_gpu_box_fit.py > gpurun_out/t33.log 2>&1 || { tail -20 gpurun_out/t33.log; exit 1; }
tail -1 gpurun_out/t33.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gf -o kt -- python3 $R/bench.py --no-secondary --no-cpu-baseline --repeats 0 --no-h2d --no-kitti --no-step-api --kstats none > $R/gpurun_out/gf.json 2> $R/gpurun_out/gf.err
python3 $R/tools/gaps.py $R/gpurun_out/gf/kt_kernel_trace.csv 60 800
python3 - $R/gpurun_out/gf/kt_kernel_trace.csv <<'PY'
import csv, sys
d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1])) if "tbd_fit" in r["Kernel_Name"])
print("tbd_fit launches", len(d), "mean us", sum(d) / len(d) / 1e3, "median", d[len(d) // 2] / 1e3)
PY
