set -u
S=tools/gpu_step.sh
B=collaborative-filtering-kafka_amd
CFK_ALS_LIB=$B/build_treg0/libcfk_als.so $S 300 dump_old.log python -u tools/dump_iteration.py --k 128 --out /tmp/old.npz || exit 1
CFK_ALS_LIB=$B/build/libcfk_als.so $S 300 dump_new.log python -u tools/dump_iteration.py --k 128 --out /tmp/new.npz || exit 1
$S 120 cmp.log python -u tools/dump_iteration.py --compare /tmp/old.npz /tmp/new.npz
rm -f /tmp/old.npz /tmp/new.npz
timeout -k 10 600 bash tools/ab_builds.sh "build build_treg0" "--k 128 --rounds 3 --variants ALS_DUAL=1 ALS_DUAL=0" 2 || exit 1
