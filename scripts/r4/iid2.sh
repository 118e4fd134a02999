#!/bin/bash
# IID learning sweep 2: larger client learning rates (averaged Adam-normalised updates of IID
# clients partly cancel, so FedAvg's effective step shrinks), 5 clients, both modes
set -o pipefail
OUT=gpurun_out/r4_iid2
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
    print('$i', r['mode'], '$cfg', r['final_accuracy'], [round(a,2) for a in r['accuracy_curve']], [round(x,2) for x in r['train_loss_curve']][-4:])"
done <<'CFGS'
lr=1e-4 adam_betas=[0.9,0.98] max_grad_norm=1.0
lr=2e-4 adam_betas=[0.9,0.98] max_grad_norm=1.0
lr=5e-5 adam_betas=[0.9,0.98] max_grad_norm=1.0 local_epochs=2
lr=1e-4 adam_betas=[0.9,0.98] max_grad_norm=1.0 lr_warmup_steps=48
CFGS
