#!/bin/bash
# attention kernel timing on the final tree (3 processes), config 5 with 3 client lanes
set -o pipefail
OUT=gpurun_out/tailchk
mkdir -p $OUT
for i in 1 2 3; do timeout -k 10 120 python -u scripts/attn_time.py > $OUT/attn_$i.log 2>&1 || { echo "attn rc=$?"; tail -5 $OUT/attn_$i.log; exit 1; }; tail -1 $OUT/attn_$i.log | cut -c1-300; done
( while sleep 30; do echo "hb $(date +%s)" >> $OUT/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 400 python -u bench.py $P --lanes 3 --steps 3 --warmup 1 > $OUT/l3.json 2> $OUT/l3.err; rc=$?
kill $HB
[ $rc -eq 0 ] || { echo "llama rc=$rc"; tail -5 $OUT/l3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/l3.json'));print('llama lanes3', round(d['value'],3), round(d['tokens_per_s']), d['hbm_peak_gb'])"
