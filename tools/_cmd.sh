mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense_lk.py tests/test_gpu_klt.py > gpurun_out/t_dense.log 2>&1; tail -3 gpurun_out/t_dense.log
timeout -k 10 200 python -u tools/probe_dense_lk.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/probe_dense_lk.py 2>&1 | grep -v amdgpu.ids
