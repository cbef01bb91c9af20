set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b22.json 2> gpurun_out/b22.err
python3 -c "
import json; d=json.loads(open('gpurun_out/b22.json').read().strip().splitlines()[-1]); print(d['value'], d['sequence']['runs_fps'], d['with_h2d']['runs_fps'], d['step_api'], d['kitti']['value'], d['roofline']['frac'])"
