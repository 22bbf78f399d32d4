# (ALS_XCD_SUBRANGES was removed after this run: rejected)
# XCD sub-ranges (ALS_XCD_SUBRANGES = S: 8 S ranges, XCD x walks ranges x, x + 8, ... in turn), k = 64 whole data
set -u
R=$(pwd); O=$R/gpurun_out/exp_subranges; mkdir -p $O
timeout -k 10 400 python3 -u tools/kbench.py --rounds 3 --variants "ALS_XCD_SUBRANGES=1" "ALS_XCD_SUBRANGES=2" "ALS_XCD_SUBRANGES=4" "ALS_XCD_RANGES=0" > $O/g1_k64.log 2>&1 || { tail -5 $O/g1_k64.log; exit 99; }
grep -v '^{' $O/g1_k64.log | grep -v '^vs' | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); d = json.loads(j)
    print('   ', v, {k: (round(d[k]['median_ms'], 3), round(d[k]['min_ms'], 3)) for k in ('movie', 'user', 'movie_reduce')})
"
echo "exp_subranges done"
