# fp64 generic path with one refinement step: every-k parity incl. 129/160/256 against the exact solution
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_k" --timeout 300 --timeout-method thread > gpurun_out/e14_everyk.log 2>&1 || { tail -30 gpurun_out/e14_everyk.log; exit 1; }
tail -1 gpurun_out/e14_everyk.log
