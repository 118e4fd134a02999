#!/bin/bash
set -o pipefail
OUT=gpurun_out/cfg2l
mkdir -p $OUT
for rep in 1 2; do for l in 6 8; do
  timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --lanes $l --steps 10 --warmup 3 > $OUT/l${l}_$rep.json 2> $OUT/l${l}_$rep.err || { echo "rc=$?"; tail -5 $OUT/l${l}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/l${l}_$rep.json'));print('server lanes=$l rep=$rep', round(d['value'],4))"
done; done
