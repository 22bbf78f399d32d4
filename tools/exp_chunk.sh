# movie-half split-row chunk size (ALS_CHUNK entries per PARTIAL task; default nnz/4096 = 24.5k at Netflix shape):
# smaller chunks = more equal task lengths (waves walk the user-sorted rows more in step) but more partial slots
set -e
for r in 1 2; do
timeout -k 10 300 python -u tools/kbench.py --k 64 --rounds 3 --variants ALS_CHUNK=24576 ALS_CHUNK=4096 ALS_CHUNK=8192 ALS_CHUNK=65536 > gpurun_out/e30_$r.log 2>&1
grep -h "median" gpurun_out/e30_$r.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('r$r', v, 'movie', round(d['movie']['median_ms'],3), 'reduce', round(d['movie_reduce']['median_ms'],3), 'user', round(d['user']['median_ms'],3), 'total', round(d['total_median_ms'],3))
"
done
