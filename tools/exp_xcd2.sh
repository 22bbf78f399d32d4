# round 2, k = 128: XCD-sliced task order (ALS_XCD_SLICE, debug build) against the plain LPT order, k = 64 / 128, whole data and shards
# (ALS_XCD_SLICE, an XCD-sliced LPT order, was removed after these runs: rejected, DESIGN.md section 7;
#  logs in profiles/r06c/xcd*_*.log)
set -u
R=$(pwd); O=$R/gpurun_out/exp_xcd2; mkdir -p $O
export CFK_ALS_LIB=$R/collaborative-filtering-kafka_amd/build_debug/libcfk_als.so
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
run g2_k128 --k 128 --shard-of 2 --variants "" "ALS_ILV_CHUNK=4096" "ALS_ILV_CHUNK=4096,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=2048,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=2048"
run g4_k128 --k 128 --shard-of 4 --variants "" "ALS_ILV_CHUNK=2048,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=4096,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=4096" "ALS_ILV_CHUNK=2048"
run g8_k128 --k 128 --shard-of 8 --variants "" "ALS_ILV_CHUNK=1024,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=2048,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=2048" "ALS_ILV_CHUNK=1024"
run g1_k128 --k 128 --variants "" "ALS_ILV_CHUNK=8192,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=4096,ALS_XCD_SLICE=1" "ALS_ILV_CHUNK=8192"
echo "exp_xcd2 done"
