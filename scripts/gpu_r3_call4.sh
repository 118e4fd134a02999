#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/taild gpurun_out/lora
timeout -k 10 120 python -u scripts/tail_diag.py > gpurun_out/taild/d.log 2>&1 || { echo "diag rc=$?"; tail gpurun_out/taild/d.log; exit 1; }
grep rep gpurun_out/taild/d.log
( while sleep 30; do echo "hb $(date +%s)" >> gpurun_out/lora/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
BCFL_LORA_TAIL=1 timeout -k 10 400 python -u bench.py $P --steps 3 --warmup 1 > gpurun_out/lora/llama_tail.json 2> gpurun_out/lora/llama_tail.err; rc=$?
kill $HB
[ $rc -eq 0 ] || { echo "llama rc=$rc"; tail -5 gpurun_out/lora/llama_tail.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/lora/llama_tail.json'));print('llama tail', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'])"
