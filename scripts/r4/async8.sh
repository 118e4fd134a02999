#!/bin/bash
# 8 ranks (one client each, the driver's 8-GPU layout) rehearsed on one GPU: async delta exchange
# + apply-on-arrival vs the round-3 same-round wait; then the IID learning sweep
set -o pipefail
OUT=gpurun_out/r4_async8
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
run() {
  tag=$1; shift
  timeout -k 10 450 python -u bench.py --gpus ${GPUS:-8} --steps 20 --warmup 5 --no-info-passing "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -20 $OUT/$tag.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$tag.json') if l.startswith('{')][-1])
pr=d['multi_rank']['per_rank']
print('$tag', round(d['value'],4), [round(p.get('lead_wait_s_total',0),2) for p in pr], d['final_accuracy'], d['accuracy_curve'], [round(sum(p['stale_rounds'])/len(p['stale_rounds']),2) for p in pr], [round(p['wait_s_total'],2) for p in pr])"
}
run n8_bounded

true
