#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then one PMC counter per pass as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass). Outputs under gpurun_out/prof_*.
#   tools/profile.sh <tag> [extra bench args...]
set -u
tag=$1; shift
export TMPDIR=/tmp
R=$(pwd)
B="--steps 3 --warmup 1 --no-cpu-baseline $*"
tools/gpu_step.sh 600 prof_${tag}_trace.log rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${tag}_trace -o run --output-format csv -- python3 $R/bench.py $B || exit 99
tools/gpu_step.sh 600 prof_${tag}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${tag}_fetch -o run --output-format csv -- python3 $R/bench.py $B || exit 99
tools/gpu_step.sh 600 prof_${tag}_write.log rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${tag}_write -o run --output-format csv -- python3 $R/bench.py $B || exit 99
