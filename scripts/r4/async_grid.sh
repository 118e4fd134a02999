#!/bin/bash
# async multi-rank learning with exchanged control variates (2 / 4 ranks on one GPU) and the
# IID stability A/B (serverless 5 clients: no clipping vs global-norm clip 1.0)
set -o pipefail
OUT=gpurun_out/r4_async
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
timeout -k 10 300 python -u benchmarks/worker_grid.py --clients 5 --modes serverless --out $OUT/grid5_base.json > $OUT/grid5_base.log 2>&1 || { echo "grid base rc=$?"; tail -20 $OUT/grid5_base.log; exit 1; }
timeout -k 10 300 python -u benchmarks/worker_grid.py --clients 5 --modes serverless --set max_grad_norm=1.0 --out $OUT/grid5_clip.json > $OUT/grid5_clip.log 2>&1 || { echo "grid clip rc=$?"; tail -20 $OUT/grid5_clip.log; exit 1; }
python -c "
import json
for t in ('base','clip'):
    d=json.load(open('$OUT/grid5_'+t+'.json'))
    for r in d['runs']:
        print(t, r['mode'], r['clients'], r['final_accuracy'], [round(a,2) for a in r['accuracy_curve']], [round(x,3) for x in r['train_loss_curve']])"
