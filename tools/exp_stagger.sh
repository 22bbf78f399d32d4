# phase-lock test: LPT vs windows alternating long/short halves (co-resident waves of different lengths)
set -e
for k in 64 128; do
timeout -k 10 300 python -u tools/kbench.py --k $k --rounds 3 --variants "ALS_TASK_ORDER=lpt" "ALS_TASK_ORDER=stagger" "ALS_TASK_ORDER=stagger:256" "ALS_TASK_ORDER=stagger:4096" > gpurun_out/e11_$k.log 2>&1
grep -h "median" gpurun_out/e11_$k.log | grep -v kbench | python3 -c "
import sys, json
for l in sys.stdin:
    v, d = l.split(' ', 1); d = json.loads(d)
    print('k$k', v, 'movie', round(d['movie']['median_ms'],3), 'user', round(d['user']['median_ms'],3))
"
done
