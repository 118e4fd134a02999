#!/bin/bash
# weight-gradient slot budget A/B (BCFL_G8_WGRAD_SLOTS) in both regimes: the driver bench (8
# clients on lanes) and the per-rank work of the 8-GPU layout (--clients 1), interleaved reps
set -o pipefail
OUT=${OUT:-gpurun_out/wgrad_slots}
mkdir -p $OUT
for rep in 1 2; do
  for sl in 16 32 64 128; do
    BCFL_G8_WGRAD_SLOTS=$sl timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-ckpt > $OUT/b8_${sl}_$rep.json 2> $OUT/b8_${sl}_$rep.err || { echo "b8 $sl rc=$?"; tail -5 $OUT/b8_${sl}_$rep.err; exit 1; }
    BCFL_G8_WGRAD_SLOTS=$sl timeout -k 10 200 python -u bench.py --clients 1 --global-test-samples 125 --steps 20 --warmup 3 --no-ckpt > $OUT/b1_${sl}_$rep.json 2> $OUT/b1_${sl}_$rep.err || { echo "b1 $sl rc=$?"; tail -5 $OUT/b1_${sl}_$rep.err; exit 1; }
    python -c "
import json
a=json.load(open('$OUT/b8_${sl}_$rep.json')); b=json.load(open('$OUT/b1_${sl}_$rep.json'))
print('slots $sl rep $rep', '8 lanes', round(a['value'],4), '1 client', round(b['value'],4))"
  done
done
