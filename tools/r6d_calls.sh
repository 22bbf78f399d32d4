set -u
tools/gpu_step.sh 1000 r6d_gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread || exit 99
tools/gpu_step.sh 300 r6d_bench.json python3 bench.py || exit 99
tools/gpu_step.sh 300 r6d_k128_g2.json python3 bench.py --k 128 --shard-of 2 --steps 20 --warmup 3 --no-cpu-baseline || exit 99
tools/gpu_step.sh 300 r6d_k128_g4.json python3 bench.py --k 128 --shard-of 4 --steps 20 --warmup 3 --no-cpu-baseline || exit 99
tools/gpu_step.sh 300 r6d_k128_g8.json python3 bench.py --k 128 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline || exit 99
