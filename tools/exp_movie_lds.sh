# movie half (k = 64 on-the-fly kernel) vs unused dynamic LDS per workgroup (debug build's ALS_DEBUG_EXTRA_LDS):
# does LDS padding change its placement / speed (round-5 occupancy sweep hinted 2.87 vs 3.00 ms at 7000 B)?
set -e
B=collaborative-filtering-kafka_amd
for r in 1 2 3; do
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py --k 64 --rounds 3 --variants ALS_DEBUG_EXTRA_LDS=0 ALS_DEBUG_EXTRA_LDS=4000 ALS_DEBUG_EXTRA_LDS=7000 ALS_DEBUG_EXTRA_LDS=12000 > gpurun_out/e22_$r.log 2>&1
grep -h "median" gpurun_out/e22_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('r$r', v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done
