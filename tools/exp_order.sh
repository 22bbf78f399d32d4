set -e
B=collaborative-filtering-kafka_amd
timeout -k 10 240 python -u tools/kbench.py --k 64 --rounds 5 --variants "ALS_TASK_ORDER=lpt" "ALS_TASK_ORDER=random" > gpurun_out/e1_k64.log 2>&1
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 240 python -u tools/kbench.py --k 64 --rounds 3 --variants "ALS_DEBUG_SKIP_SOLVE=1" "ALS_DEBUG_SKIP_SOLVE=1,ALS_TASK_ORDER=random" > gpurun_out/e1_k64_gram.log 2>&1
timeout -k 10 300 python -u tools/kbench.py --k 128 --rounds 3 --variants "ALS_TASK_ORDER=lpt" "ALS_TASK_ORDER=random" > gpurun_out/e1_k128.log 2>&1
grep -h total_median gpurun_out/e1_*.log | cut -c1-600
