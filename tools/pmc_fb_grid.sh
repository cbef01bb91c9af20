set -e
root=$(pwd); cd /tmp; export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1)); out=$root/gpurun_out/fbpmc$i; mkdir -p $out
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out -o pmc -- python3 $root/tools/bench_farneback.py --pairs 2 --warmup 1 --flags 0 > $out/bench.json 2> $out/err.txt
  f=$(find $out -name 'pmc_counter_collection.csv' | head -1)
  python3 $root/tools/pmc_by_grid.py $f fb_iter > $out/by_grid.txt
done
