# k = 64 shards: shorter interleave chunks (ALS_ILV_CHUNK, debug build) with and without XCD ranges, against the
# default contiguous plan (kbench, one process per G)
set -u
R=$(pwd); O=$R/gpurun_out/exp_shard_ranges; mkdir -p $O
export CFK_ALS_LIB=$R/collaborative-filtering-kafka_amd/build_debug/libcfk_als.so
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
run g2 --shard-of 2 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=4096,ALS_XCD_RANGES=1" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=4096,ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=2048,ALS_XCD_RANGES=1"
run g4 --shard-of 4 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=2048,ALS_XCD_RANGES=1" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=1024,ALS_XCD_RANGES=1"
run g8 --shard-of 8 --variants "ALS_XCD_RANGES=0" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=1024,ALS_XCD_RANGES=1" "ALS_INTERLEAVE=1,ALS_ILV_CHUNK=512,ALS_XCD_RANGES=1"
echo "exp_shard_ranges done"
