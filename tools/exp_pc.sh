# pipelined pre-split launch: parity subset, then kbench A/B against the one-kernel launch at k = 64 and 128
set -e
B=collaborative-filtering-kafka_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_k or chunked or short_rows or f64_parity or split_rows" --timeout 120 --timeout-method thread > gpurun_out/e5_parity.log 2>&1 || { tail -30 gpurun_out/e5_parity.log; exit 1; }
tail -2 gpurun_out/e5_parity.log
timeout -k 10 300 python -u tools/kbench.py --k 64 --rounds 5 --variants "ALS_PC=0" "ALS_PC=1" > gpurun_out/e5_k64.log 2>&1
grep -h "^vs\|^ALS" gpurun_out/e5_k64.log | cut -c1-400
timeout -k 10 300 python -u tools/kbench.py --k 128 --rounds 3 --variants "ALS_PC=0" "ALS_PC=1" > gpurun_out/e5_k128.log 2>&1
grep -h "^vs\|^ALS" gpurun_out/e5_k128.log | cut -c1-400
