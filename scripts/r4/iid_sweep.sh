#!/bin/bash
# IID serverless-5 learning sweep (20 rounds x 4 local steps): lr / beta2 / clipping / warm-up
set -o pipefail
OUT=gpurun_out/r4_iid
mkdir -p $OUT
i=0
while read -r cfg; do
  i=$((i+1))
  sets=""; for kv in $cfg; do sets="$sets --set $kv"; done
  timeout -k 10 150 python -u benchmarks/worker_grid.py --clients 5 --modes serverless server $sets --out $OUT/g$i.json > $OUT/g$i.log 2>&1 || { echo "g$i rc=$?"; tail -20 $OUT/g$i.log; exit 1; }
  python -c "
import json
d=json.load(open('$OUT/g$i.json'))
for r in d['runs']:
    print('$i', '$cfg', r['final_accuracy'], [round(a,2) for a in r['accuracy_curve']], [round(x,2) for x in r['train_loss_curve']][-6:])"
done <<'CFGS'
outer_momentum=0.9
outer_momentum=0.9 outer_lr=0.7
outer_momentum=0.9 max_grad_norm=1.0 adam_betas=[0.9,0.98]
adam_betas=[0.9,0.98] lr=5e-05 max_grad_norm=1.0
outer_momentum=0.8 lr=3e-05 max_grad_norm=1.0
CFGS
