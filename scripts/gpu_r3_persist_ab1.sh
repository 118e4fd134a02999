#!/bin/bash
# one-client round (per-rank work of the 8-GPU layout): persistent 8-phase grids off / on, 3
# interleaved reps each, plus a 2-rank same-round-mix check after the bounded-wait change
set -o pipefail
OUT=gpurun_out/pab
mkdir -p $OUT
for rep in 1 2 3; do for v in 0 1; do
  BCFL_G8_PERSIST=$v timeout -k 10 200 python -u bench.py --clients 1 --global-test-samples 125 --steps 10 --warmup 3 > $OUT/p${v}_$rep.json 2> $OUT/p${v}_$rep.err || { echo "rc=$?"; tail -5 $OUT/p${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/p${v}_$rep.json'));print('persist=$v rep=$rep', round(d['value'],4))" | tee -a $OUT/ab.log
done; done
