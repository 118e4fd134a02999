#!/bin/bash
# delta exchange (cumulative own updates, applied once) + exchanged control variates: 2 / 4 ranks
# on one GPU, the driver's bench config; then the IID serverless-5 learning-rate sweep
set -o pipefail
OUT=gpurun_out/r4_async2
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 20 --warmup 5 --no-info-passing > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -20 $OUT/n$n.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/n$n.json') if l.startswith('{')][-1])
pr=d['multi_rank']['per_rank']
print('$n', round(d['value'],4), d['final_accuracy'], d['config']['gossip_mix'], [p['stale_rounds'][-3:] for p in pr], [round(p['wait_s_total'],3) for p in pr])"
done
unset BCFL_DIST_BACKEND
for cfg in "lr=5e-05" "lr=5e-05 max_grad_norm=1.0" "lr=0.0001 max_grad_norm=1.0" "drift_correction=scaffold"; do
  tag=$(echo $cfg | tr ' =' '__')
  sets=""; for kv in $cfg; do sets="$sets --set $kv"; done
  timeout -k 10 300 python -u benchmarks/worker_grid.py --clients 5 --modes serverless $sets --out $OUT/grid5_$tag.json > $OUT/grid5_$tag.log 2>&1 || { echo "grid $tag rc=$?"; tail -20 $OUT/grid5_$tag.log; exit 1; }
  python -c "
import json
d=json.load(open('$OUT/grid5_$tag.json'))
for r in d['runs']:
    print('$tag', r['mode'], r['clients'], r['final_accuracy'], [round(a,2) for a in r['accuracy_curve']], [round(x,3) for x in r['train_loss_curve']][-5:])"
done
