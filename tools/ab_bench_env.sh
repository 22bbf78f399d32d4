# bench.py A/B of an engine env setting on one box: "<envA>" "<envB>" [ROUNDS] [bench args...], runs interleaved
set -u
A=$1; B=$2; rounds=${3:-2}; shift 3
mkdir -p gpurun_out/ab_env
for r in $(seq 1 $rounds); do
    for v in "$A" "$B"; do
        tag=$(echo "$v" | tr -c 'A-Za-z0-9' '_')
        env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab_env/${tag}_$r.json 2>&1 || exit 99
        python3 -c "
import json, sys
d = json.loads([l for l in open('gpurun_out/ab_env/${tag}_$r.json') if l.startswith('{')][-1])
pl = d['roofline']['per_launch']
print('$v', 'round $r', round(d['ms_per_step'], 4), {h: (round(v['avg_launch_ms'], 3), round(v['reduce_launch_ms'], 3)) for h, v in pl.items()})
"
    done
done
