# solver phase breakdown of the pipelined launch (debug build)
set -e
B=collaborative-filtering-kafka_amd
for k in 64 128; do
CFK_ALS_LIB=$B/build_debug/libcfk_als.so timeout -k 10 200 python -u tools/kbench.py --k $k --rounds 1 --variants "ALS_PC=1" > gpurun_out/e10_$k.log 2>&1
echo "k$k $(grep -h "^pc_stats" gpurun_out/e10_$k.log | cut -c1-900)"
done
