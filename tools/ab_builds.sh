#!/bin/bash
# A/B of library builds (collaborative-filtering-kafka_amd/<build>/libcfk_als.so) on one box: a parity smoke of
# every build (the every-k oracle test at the given k), then kbench in separate processes, builds interleaved
# over ROUNDS rounds. Prints one summary line per (round, build).
#   tools/ab_builds.sh "<build dirs>" "<kbench args>" [ROUNDS] [pytest -k expression]
set -u
B=collaborative-filtering-kafka_amd
builds=$1; kargs=$2; rounds=${3:-2}; kexpr=${4:-}
mkdir -p gpurun_out
if [ -n "$kexpr" ]; then
    for v in $builds; do
        CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q \
            -k "$kexpr" --timeout 200 --timeout-method thread > gpurun_out/ab_test_$v.log 2>&1
        rc=$?
        echo "$v parity: rc=$rc $(tail -1 gpurun_out/ab_test_$v.log)"
        [ $rc -ge 124 ] && exit 99
    done
fi
for r in $(seq 1 $rounds); do
    for v in $builds; do
        CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 300 python -u tools/kbench.py $kargs > gpurun_out/ab_${v}_$r.log 2>&1 || exit 99
        tail -1 gpurun_out/ab_${v}_$r.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['kbench']
for var, x in d.items():
    print('$v', 'round $r', var, {k: round(x[k]['median_ms'], 3) for k in ('movie', 'user', 'movie_reduce', 'user_reduce')}, round(x['total_median_ms'], 3))
"
    done
done
