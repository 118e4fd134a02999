#!/bin/bash
# config 5 A/B on one box: LoRA low-rank products on the 8-phase GEMM vs the library (both with
# the tail-segment base GEMMs); then the worker grid after the lanes' local evaluation
set -o pipefail
mkdir -p gpurun_out/lora gpurun_out/r3g
( while sleep 30; do echo "hb $(date +%s)" >> gpurun_out/lora/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
for v in 1 0 1; do
  BCFL_LORA_G8=$v timeout -k 10 400 python -u bench.py $P --steps 3 --warmup 1 > gpurun_out/lora/ab_$v.json 2> gpurun_out/lora/ab_$v.err || { kill $HB; echo "llama $v failed"; tail -5 gpurun_out/lora/ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lora/ab_$v.json'));print('llama g8skinny=$v', round(d['value'],3), round(d['tokens_per_s']))" | tee -a gpurun_out/lora/ab.log
done
kill $HB
timeout -k 10 900 python -u benchmarks/worker_grid.py --out gpurun_out/r3g/worker_grid.json > gpurun_out/r3g/grid.log 2>&1 || { echo "grid rc=$?"; tail -20 gpurun_out/r3g/grid.log; exit 1; }
tail -6 gpurun_out/r3g/grid.log | cut -c1-200
