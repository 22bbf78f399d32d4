# XCD range pieces of the interleaved half (ALS_XCD_RANGES) against the plain interleave, k = 64 / 128, whole data and
# shards (kbench, one process per configuration, variants interleaved), then the interleave parity tests
set -u
R=$(pwd); O=$R/gpurun_out/exp_ranges; mkdir -p $O
run() {
    local n=$1; shift
    timeout -k 10 300 python3 -u tools/kbench.py --rounds 3 "$@" > $O/$n.log 2>&1
    local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$n.log; exit 99; }
    grep -v '^{' $O/$n.log | grep -v '^vs' | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); d = json.loads(j)
    print('   ', v, {k: round(d[k]['median_ms'], 3) for k in ('movie', 'user', 'movie_reduce')})
"
    return 0
}
run g1_k64 --variants "ALS_XCD_RANGES=0" "ALS_XCD_RANGES=1" "ALS_XCD_RANGES=1,ALS_XCD_RANGE_MIN=4096" "ALS_XCD_RANGES=1,ALS_XCD_RANGE_MIN=2048"   # (ALS_XCD_RANGE_MIN: removed after this run)
run g2_k64 --shard-of 2 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=1"
run g4_k64 --shard-of 4 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=1"
run g1_k128 --k 128 --variants "ALS_XCD_RANGES=0" "ALS_XCD_RANGES=1"
run g2_k128 --k 128 --shard-of 2 --variants "ALS_XCD_RANGES=0" "ALS_XCD_RANGES=1"
timeout -k 10 600 python -u -m pytest tests/test_gpu_interleave.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"; tail -6 $O/tests.log
echo "exp_ranges done"
