# pipelined k = 64 launch with 8 / 10 Gram waves of 16 (build_pc8, build_pc10; 6 hand-off slots) vs the one-kernel
# launch: parity of the pc8 path, then kbench (ALS_PC=0 = one-kernel, ALS_PC=1 = pipelined) in interleaved rounds
set -e
B=collaborative-filtering-kafka_amd
ALS_PC=1 CFK_ALS_LIB=$B/build_pc8/libcfk_als.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_k or determinism or short_rows" --timeout 120 --timeout-method thread > gpurun_out/e21_parity.log 2>&1 || { tail -30 gpurun_out/e21_parity.log; exit 1; }
tail -1 gpurun_out/e21_parity.log
for r in 1 2; do for v in build_pc8 build_pc10; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 64 --rounds 3 --variants ALS_PC=0 ALS_PC=1 > gpurun_out/e21_${v}_$r.log 2>&1
grep -h "median" gpurun_out/e21_${v}_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v r$r', v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done; done
