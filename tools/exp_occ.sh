# occupancy sweep of the pre-split kernels (debug build: unused LDS per workgroup; Gram-only vs full), from one factor snapshot
set -e
B=collaborative-filtering-kafka_amd
summ() { grep -h "median" $1 | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print(v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3))
"; }
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py --k 64 --rounds 3 --variants \
  "ALS_DEBUG_SKIP_SOLVE=1" "ALS_DEBUG_SKIP_SOLVE=1,ALS_DEBUG_EXTRA_LDS=7000" "ALS_DEBUG_SKIP_SOLVE=1,ALS_DEBUG_EXTRA_LDS=20000" \
  "ALS_DEBUG_SKIP_SOLVE=0" "ALS_DEBUG_SKIP_SOLVE=0,ALS_DEBUG_EXTRA_LDS=7000" "ALS_DEBUG_SKIP_SOLVE=0,ALS_DEBUG_EXTRA_LDS=20000" > gpurun_out/e4_occ.log 2>&1
summ gpurun_out/e4_occ.log
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py --k 128 --rounds 3 --variants \
  "ALS_DEBUG_SKIP_SOLVE=1" "ALS_DEBUG_SKIP_SOLVE=0" > gpurun_out/e4_128.log 2>&1
summ gpurun_out/e4_128.log
