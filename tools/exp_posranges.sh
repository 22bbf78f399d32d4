# (ALS_XCD_RANGES=2, position ranges, was removed after this run: rejected)
# XCD ranges by block position in the row (ALS_XCD_RANGES=2) vs by opposite slot (=1) vs the defaults, k = 64 shards
set -u
R=$(pwd); O=$R/gpurun_out/exp_posranges; mkdir -p $O
run() {
    local n=$1; shift
    timeout -k 10 400 python3 -u tools/kbench.py --rounds 3 "$@" > $O/$n.log 2>&1
    local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$n.log; exit 99; }
    grep -v '^{' $O/$n.log | grep -v '^vs' | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); d = json.loads(j)
    print('   ', v, {k: (round(d[k]['median_ms'], 3), round(d[k]['min_ms'], 3)) for k in ('movie', 'user', 'movie_reduce')})
"
    return 0
}
run g1_k64 --variants "ALS_XCD_RANGES=1" "ALS_XCD_RANGES=2"
run g2_k64 --shard-of 2 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=2" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=0"
run g4_k64 --shard-of 4 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=2"
run g8_k64 --shard-of 8 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_XCD_RANGES=2"
echo "exp_posranges done"
