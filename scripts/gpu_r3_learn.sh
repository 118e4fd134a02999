#!/bin/bash
# multi-rank learning on one GPU: the driver's bench config (20 timed + 5 warmup rounds) at 2 and
# 4 ranks (gloo collectives, hipIpc mailboxes between the rank processes)
set -o pipefail
OUT=gpurun_out/learn
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 20 --warmup 5 > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -20 $OUT/n$n.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/n$n.json') if l.startswith('{')][-1])
print('$n', round(d['value'],4), d['final_accuracy'], d['final_accuracy_scope'][:60], d['multi_rank']['per_rank'][0]['mixed'])"
done
