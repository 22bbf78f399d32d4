# is the pivot-gated refinement step a real share of the k = 64 user half? (debug build: refinement knobs)
set -e
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py --k 64 --rounds 3 --variants \
  "ALS_DEBUG_SKIP_REFINE=0" "ALS_DEBUG_SKIP_REFINE=1" "ALS_REFINE_MIN_PIVOT=0" "ALS_REFINE_MIN_PIVOT=2" > gpurun_out/e3_ref.log 2>&1
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py --k 128 --rounds 3 --variants \
  "ALS_DEBUG_SKIP_REFINE=0" "ALS_DEBUG_SKIP_REFINE=1" > gpurun_out/e3_ref128.log 2>&1
for f in gpurun_out/e3_ref.log gpurun_out/e3_ref128.log; do
grep -h "median" $f | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print(v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3))
"; done
