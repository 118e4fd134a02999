#!/bin/bash
# 8-client bench: client lanes 8 / 6 / 4, interleaved, 2 reps
set -o pipefail
OUT=gpurun_out/lab
mkdir -p $OUT
for rep in 3 4; do for l in 6 8 7; do
  timeout -k 10 200 python -u bench.py --lanes $l --steps 12 --warmup 3 --no-info-passing > $OUT/l${l}_$rep.json 2> $OUT/l${l}_$rep.err || { echo "rc=$?"; tail -5 $OUT/l${l}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/l${l}_$rep.json'));print('lanes=$l rep=$rep', round(d['value'],4))" | tee -a $OUT/ab.log
done; done
