# bench.py A/B of two library builds on one box: "<build dir A>" "<build dir B>" [ROUNDS] [bench args...]
set -u
A=$1; B=$2; rounds=${3:-2}; shift 3
mkdir -p gpurun_out/ab_libs
for r in $(seq 1 $rounds); do
    for v in "$A" "$B"; do
        CFK_ALS_LIB=collaborative-filtering-kafka_amd/$v/libcfk_als.so timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab_libs/${v}_$r.json 2>&1 || exit 99
        python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ab_libs/${v}_$r.json') if l.startswith('{')][-1])
pl = d['roofline']['per_launch']
print('$v', 'round $r', round(d['ms_per_step'], 4), {h: (round(v['avg_launch_ms'], 3), round(v['reduce_launch_ms'], 3)) for h, v in pl.items()})
"
    done
done
