set -u
B=collaborative-filtering-kafka_amd
tools/gpu_step.sh 300 t_cr.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q --timeout 250 --timeout-method thread -k "every_k or extreme or split or determinism or fullscale or full" || exit 1
grep -q "passed" gpurun_out/t_cr.log || exit 1
tools/gpu_step.sh 200 d1.log python tools/dump_iteration.py --k 64 --out gpurun_out/cr1.npz || exit 1
CFK_ALS_LIB=$B/build_cr0/libcfk_als.so tools/gpu_step.sh 200 d0.log python tools/dump_iteration.py --k 64 --out gpurun_out/cr0.npz || exit 1
python tools/dump_iteration.py --compare gpurun_out/cr0.npz gpurun_out/cr1.npz
tools/ab_builds.sh "build build_cr0" "--rounds 5" 3
