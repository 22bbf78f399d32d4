# k = 128 pre-split Gram with the LDS-DMA two blocks ahead (build_db) vs one (build): parity, then interleaved kbench
set -e
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_db/libcfk_als.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_k and (65 or 96 or 127 or 128)" --timeout 120 --timeout-method thread > gpurun_out/e15_parity.log 2>&1 || { tail -30 gpurun_out/e15_parity.log; exit 1; }
tail -1 gpurun_out/e15_parity.log
for r in 1 2; do for v in build build_db; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 128 --rounds 3 > gpurun_out/e15_${v}_$r.log 2>&1
grep -h "median" gpurun_out/e15_${v}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v r$r', 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done
