#!/bin/bash
# One GPU call: bitwise A/B of library builds on one Netflix-shape iteration (k given, default 64) against the first build, the
# GPU parity subset that exercises the pre-split user half on every other build, and interleaved kbench rounds of
# all builds.
#   tools/ab_iteration.sh "<old build dir> <new build dir> [more builds...]" [rounds] [k]
set -u
B=collaborative-filtering-kafka_amd
builds=$1; rounds=${2:-3}; K=${3:-64}
old=${builds%% *}
mkdir -p gpurun_out
for v in $builds; do
    CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 300 python -u tools/dump_iteration.py --k $K --out /tmp/it_$v.npz \
        > gpurun_out/dump_$v.log 2>&1 || { tail -5 gpurun_out/dump_$v.log; exit 99; }
    [ "$v" != "$old" ] && python tools/dump_iteration.py --compare /tmp/it_$old.npz /tmp/it_$v.npz \
        | sed "s/^/$v vs $old: /" | tee -a gpurun_out/ab_compare.log
done
for v in $builds; do
    [ "$v" == "$old" ] && continue
    CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
        tests/test_gpu_integrity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
        -k "every_k or presplit or short_rows or chunked or determinism or full_run or deterministic or extreme or gram_variants or sharded" \
        > gpurun_out/ab_parity_$v.log 2>&1
    rc=$?
    echo "$v parity rc=$rc: $(tail -1 gpurun_out/ab_parity_$v.log)"
    [ $rc -ge 124 ] && exit 99
done
bash tools/ab_builds.sh "$builds" "--k $K --rounds 3" "$rounds"
