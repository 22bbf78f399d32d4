# A/B of the pre-split Gram in scaled units + zero-C first block (build) against HEAD (build_base), then the
# parity files of the new build
set -u
tools/ab_builds.sh "build_base build" "--rounds 3" 3 "every_k or presplit or guard or refine" > gpurun_out/r6e_ab.log 2>&1
rc=$?; cat gpurun_out/r6e_ab.log; [ $rc -ne 0 ] && exit 99
tools/gpu_step.sh 900 r6e_parity.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_interleave.py tests/test_gpu_fullscale.py -m gpu -v --timeout 600 --timeout-method thread || exit 99
