#!/bin/bash
# 4 ranks on one GPU: delta exchange default vs longer liveness vs same-round (r3) for reference
set -o pipefail
OUT=gpurun_out/r4_async3
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
run() {
  tag=$1; shift
  timeout -k 10 400 python -u bench.py --gpus ${GPUS:-4} --steps 20 --warmup 5 --no-info-passing "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -20 $OUT/$tag.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$tag.json') if l.startswith('{')][-1])
pr=d['multi_rank']['per_rank']
print('$tag', round(d['value'],4), d['final_accuracy'], d['accuracy_curve'], [round(sum(p['stale_rounds'])/len(p['stale_rounds']),2) for p in pr])"
}
GPUS=2 run n2_delta
run n4_delta
run n4_same --set drift_same_round_mix=true
run n4_nomid --set gossip_apply_on_arrival=false
