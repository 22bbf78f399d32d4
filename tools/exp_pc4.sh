# pipelined launch cycle accounting (debug build): where do the Gram and solver waves spend their cycles
set -e
B=collaborative-filtering-kafka_amd
for k in 64 128; do
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k $k --rounds 2 --variants "ALS_PC=1" > gpurun_out/e8_$k.log 2>&1
grep -h "^pc_stats\|^ALS" gpurun_out/e8_$k.log | cut -c1-400
done
