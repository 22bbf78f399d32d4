set -u
tools/gpu_step.sh 1000 r6f_gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread || exit 99
bash tools/profile_round.sh r06d || exit 99
