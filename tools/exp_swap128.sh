# KP = 128 sweep column broadcasts by lane swaps (build_sw128, CFK_COL_SWAP=128) vs ds_bpermute (product):
# parity subset, then interleaved kbench at k = 128
set -e
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_sw128/libcfk_als.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_k or determinism or short_rows" --timeout 120 --timeout-method thread > gpurun_out/e20_parity.log 2>&1 || { tail -30 gpurun_out/e20_parity.log; exit 1; }
tail -1 gpurun_out/e20_parity.log
for r in 1 2 3; do for v in build build_sw128; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 128 --rounds 3 > gpurun_out/e20_${v}_$r.log 2>&1
grep -h "median" gpurun_out/e20_${v}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v k128 r$r', 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done
