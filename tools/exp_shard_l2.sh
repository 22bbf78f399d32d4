# L2 hit share of one rank's k = 64 movie half at G = 2 (and of the whole-data half for comparison): contiguous plan,
# interleave, interleave + XCD ranges (one TCC pass over kbench; dispatches told apart by kernel and grid size)
set -u
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/exp_shard_l2; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$O/g2" -o run --output-format csv -- python3 "$R/tools/kbench.py" --rounds 1 --shard-of 2 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=1" > $O/g2.log 2>&1 || { echo "g2 pass failed"; tail -5 $O/g2.log; exit 99; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$O/g1" -o run --output-format csv -- python3 "$R/tools/kbench.py" --rounds 1 --variants "ALS_XCD_RANGES=0" "ALS_XCD_RANGES=1" > $O/g1.log 2>&1 || { echo "g1 pass failed"; tail -5 $O/g1.log; exit 99; }
echo "exp_shard_l2 done"
