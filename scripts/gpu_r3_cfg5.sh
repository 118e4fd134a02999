#!/bin/bash
# config 5 record on the final defaults (batch 32, 2 lanes, tail-segment LoRA, library skinny
# products): 5 timed + 1 warmup rounds
set -o pipefail
OUT=gpurun_out/cfg5
mkdir -p $OUT
( while sleep 30; do echo "hb $(date +%s)" >> $OUT/hb.log; done ) & HB=$!
timeout -k 10 500 python -u bench.py --model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100 --steps 5 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err; rc=$?
kill $HB
[ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('cfg5', round(d['value'],3), round(d['tokens_per_s']), d['hbm_peak_gb'], d['config']['global_batch'], d['exchange'])"
