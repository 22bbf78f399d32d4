set -u
tools/gpu_step.sh 600 t_all.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/t_all.log && ! grep -q "failed" gpurun_out/t_all.log || exit 1
ALS_SPLIT_WAVES=3 tools/gpu_step.sh 300 t_sw3.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q --timeout 250 --timeout-method thread -k "every_k or extreme or split or determinism or fullscale or full" || exit 1
grep -q " passed" gpurun_out/t_sw3.log && ! grep -q "failed" gpurun_out/t_sw3.log || exit 1
tools/gpu_step.sh 300 kb.log python tools/kbench.py --variants "ALS_SPLIT_WAVES=2" "ALS_SPLIT_WAVES=3" "ALS_MFMA_WAVES=2" --rounds 7 || exit 1
tools/gpu_step.sh 200 bench64.log python bench.py || exit 1
