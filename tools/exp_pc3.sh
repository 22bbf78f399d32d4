# pipelined launch with per-XCD chunked task streams: A/B against the one-kernel launch; Gram-wave count at k = 64
set -e
B=collaborative-filtering-kafka_amd
summ() { grep -h "median" $1 | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('$2', v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3))
"; grep -h "^vs" $1 | cut -c1-250; }
for v in build build_pc build_pe; do
  CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k 64 --rounds 3 --variants "ALS_PC=0" "ALS_PC=1" > gpurun_out/e7_${v}_64.log 2>&1
  summ gpurun_out/e7_${v}_64.log "$v k64"
done
timeout -k 10 200 python -u tools/kbench.py --k 128 --rounds 3 --variants "ALS_PC=0" "ALS_PC=1" > gpurun_out/e7_128.log 2>&1
summ gpurun_out/e7_128.log "k128"
