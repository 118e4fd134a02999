#!/bin/bash
# IID serverless-5 learning sweep (20 rounds x 4 local steps): lr / beta2 / clipping / warm-up
set -o pipefail
OUT=gpurun_out/r4_iid
mkdir -p $OUT
i=0
while read -r cfg; do
  i=$((i+1))
  sets=""; for kv in $cfg; do sets="$sets --set $kv"; done
  timeout -k 10 200 python -u benchmarks/worker_grid.py --clients 5 --modes serverless $sets --out $OUT/g$i.json > $OUT/g$i.log 2>&1 || { echo "g$i rc=$?"; tail -20 $OUT/g$i.log; exit 1; }
  python -c "
import json
d=json.load(open('$OUT/g$i.json'))
for r in d['runs']:
    print('$i', '$cfg', r['final_accuracy'], [round(a,2) for a in r['accuracy_curve']], [round(x,2) for x in r['train_loss_curve']][-6:])"
done <<'CFGS'
adam_betas=[0.9,0.98] lr=5e-05 max_grad_norm=1.0
adam_betas=[0.9,0.98] lr=0.0001 max_grad_norm=1.0 lr_warmup_steps=40
adam_betas=[0.9,0.98] lr=3e-05 max_grad_norm=1.0
lr=5e-05 max_grad_norm=0.5
adam_betas=[0.9,0.95] lr=5e-05 max_grad_norm=1.0
adam_betas=[0.9,0.98] lr=5e-05 max_grad_norm=1.0 synthetic_signal=16.0
CFGS
