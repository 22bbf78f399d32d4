# final check of the round-6 tree: the -m gpu suite, then the default bench line
set -u
tools/gpu_step.sh 1000 r6g_gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread || exit 99
tools/gpu_step.sh 300 r6g_bench.json python3 bench.py || exit 99
