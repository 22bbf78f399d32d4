set -u
B=collaborative-filtering-kafka_amd
tools/gpu_step.sh 300 t.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/t.log && ! grep -q "failed" gpurun_out/t.log || exit 1
tools/gpu_step.sh 300 d1.log python tools/dump_iteration.py --k 64 --out gpurun_out/new.npz || exit 1
CFK_ALS_LIB=$B/build_prev/libcfk_als.so tools/gpu_step.sh 200 d0.log python tools/dump_iteration.py --k 64 --out gpurun_out/old.npz || exit 1
python tools/dump_iteration.py --compare gpurun_out/old.npz gpurun_out/new.npz
rm -f gpurun_out/*.npz
tools/ab_builds.sh "build build_prev" "--variants ALS_MFMA_WAVES=0 --rounds 5" 4
