#!/bin/bash
# A/B of library builds on the split-row stress (tools/split_diag.py) and bench.py, one box:
#   tools/variants_split.sh "<build dirs>" [reps]
B=collaborative-filtering-kafka_amd
export REPS=${2:-300} READ_U=1
for v in $1; do
  CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 300 python -u tools/split_diag.py > gpurun_out/diag_$v.log 2>&1 || exit $?
  echo "$v: $(tail -1 gpurun_out/diag_$v.log | cut -c1-200)"
done
for v in $1; do
  CFK_ALS_LIB=$B/$v/libcfk_als.so timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_$v.log 2>&1 || exit $?
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": {[^}]*}' gpurun_out/bench_$v.log | tr '\n' ' ')"
done
