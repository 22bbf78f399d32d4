#!/bin/bash
# One GPU call: A/B of two library builds (kbench k = 64 and 128, interleaved rounds), the full -m gpu suite on the
# product build, then one default bench line + a rocprofv3 kernel trace of a short bench. Every step under its own
# time limit (tools/gpu_step.sh stops the call on a fault / abort / timeout).
#   tools/gpu_call_ab_tests.sh "<build A> <build B>" <tag>
set -u
builds=$1; tag=$2
export TMPDIR=/tmp
tools/gpu_step.sh 300 ab64_$tag.log tools/ab_builds.sh "$builds" "--k 64" 2 || exit 99
tools/gpu_step.sh 300 ab128_$tag.log tools/ab_builds.sh "$builds" "--k 128" 2 || exit 99
tools/gpu_step.sh 600 pytest_gpu_$tag.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
tools/gpu_step.sh 200 bench_$tag.json python bench.py || exit 99
mkdir -p gpurun_out/trace_$tag
tools/gpu_step.sh 200 trace_$tag.log rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline || exit 99
echo "call $tag done"
