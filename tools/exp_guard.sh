# pre-split range guard: its GPU tests, then the cost of the guarded fallback launch (build = guard, build_x = none)
set -e
B=collaborative-filtering-kafka_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_parity.py -m gpu -x -q -k "guard or extreme or every_k or split_rows or short_rows" --timeout 150 --timeout-method thread > gpurun_out/e13_tests.log 2>&1 || { tail -40 gpurun_out/e13_tests.log; exit 1; }
tail -1 gpurun_out/e13_tests.log
for r in 1 2; do for v in build build_x; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 64 --rounds 3 > gpurun_out/e13_${v}_$r.log 2>&1
grep -h "median" gpurun_out/e13_${v}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v r$r', 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done
