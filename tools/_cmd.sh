mkdir -p gpurun_out
bash tools/profile_round.sh r05 > gpurun_out/prof_r05.log 2>&1 || { tail -5 gpurun_out/prof_r05.log; exit 1; }
