# device code with the compiler wave-priority pass (-amdgpu-set-wave-priority, build_wp) vs the product: the whole
# -m gpu suite on build_wp, then interleaved kbench at k = 64 / 128 (not the product build)
set -e
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_wp/libcfk_als.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e29_tests.log 2>&1 || { tail -30 gpurun_out/e29_tests.log; exit 1; }
tail -1 gpurun_out/e29_tests.log
for k in 64 128; do for r in 1 2 3; do for v in build build_wp; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k $k --rounds 3 > gpurun_out/e29_${v}_${k}_$r.log 2>&1
grep -h "median" gpurun_out/e29_${v}_${k}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v k$k r$r', 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done; done
