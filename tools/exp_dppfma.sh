# sweep row broadcasts fused into v_fmac_f32_dpp (build_df, CFK_SWEEP_DPPFMA=1) vs the product: parity subset, then
# interleaved kbench at k = 64 / 128
set -e
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_df/libcfk_als.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_integrity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e18_parity.log 2>&1 || { tail -30 gpurun_out/e18_parity.log; exit 1; }
tail -1 gpurun_out/e18_parity.log
for k in 64 128; do for r in 1 2 3; do for v in build build_df; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k $k --rounds 3 > gpurun_out/e18_${v}_${k}_$r.log 2>&1
grep -h "median" gpurun_out/e18_${v}_${k}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v k$k r$r', 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done; done
