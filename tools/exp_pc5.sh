# sweep column broadcasts by lane swaps (shorter latency) vs ds_bpermute: solver cycles per solve (debug) and timing
set -e
B=collaborative-filtering-kafka_amd
for k in 64 128; do
for v in build_debug build_dbg_sw; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k $k --rounds 2 --variants "ALS_PC=1" > gpurun_out/e9_${v}_$k.log 2>&1
echo "$v k$k $(grep -h "^pc_stats" gpurun_out/e9_${v}_$k.log | cut -c1-400)"
done; done
for v in build build_sw; do
CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 64 --rounds 3 --variants "ALS_PC=0" "ALS_PC=1" > gpurun_out/e9_${v}_t64.log 2>&1
grep -h "median" gpurun_out/e9_${v}_t64.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$v', v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3))
"
done
