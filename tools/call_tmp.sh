set -u
ALS_MFMA_WAVES=2 tools/gpu_step.sh 200 d0.log python tools/dump_iteration.py --k 64 --out gpurun_out/w2.npz || exit 1
tools/gpu_step.sh 200 d1.log python tools/dump_iteration.py --k 64 --out gpurun_out/w3.npz || exit 1
python tools/dump_iteration.py --compare gpurun_out/w2.npz gpurun_out/w3.npz
rm -f gpurun_out/*.npz
