# L1 (vector cache) reuse of the gathers: the hot-row gather microbenchmark, then one TCP counter pass over it
# (calibration: requests per wave-instruction of a known pattern) and one over the k = 64 bench launches
set -u
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/prof_l1; mkdir -p $O
timeout -k 10 120 ./tools/gather_bench > $O/gather_bench.log 2>&1 || { echo "gather_bench failed"; tail -5 $O/gather_bench.log; exit 99; }
cat $O/gather_bench.log
C="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -d "$O/gb" -o run --output-format csv -- ./tools/gather_bench > $O/gb.log 2>&1 || { echo "gb pass failed"; tail -5 $O/gb.log; exit 99; }
timeout -s KILL 180 rocprofv3 --pmc $C -d "$O/bench" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench pass failed"; tail -5 $O/bench.log; exit 99; }
echo "exp_l1 done"
