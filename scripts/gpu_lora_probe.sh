#!/bin/bash
# LoRA tail-segment GEMMs at the Llama-3-8B shapes (numerics + timings), then config 5.
set -o pipefail
OUT=gpurun_out/lora
mkdir -p $OUT
timeout -k 10 120 python -u scripts/lora_tail_bench.py 8192 2>&1 | tee $OUT/tail.log || { echo "tail rc=$?"; exit 1; }
( while sleep 30; do echo "hb $(date +%s)" >> $OUT/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 300 python -u bench.py $P --steps 3 --warmup 1 > $OUT/llama.json 2> $OUT/llama.err; rc=$?
kill $HB
[ $rc -eq 0 ] || { echo "llama rc=$rc"; tail -20 $OUT/llama.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/llama.json'));print('llama', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'], d['config'])"
