#!/bin/bash
# config 5: 4 client lanes vs 2, then a kernel summary of the 2-lane round (tail-segment LoRA)
set -o pipefail
mkdir -p gpurun_out/lora
( while sleep 30; do echo "hb $(date +%s)" >> gpurun_out/lora/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 400 python -u bench.py $P --lanes 4 --steps 3 --warmup 1 > gpurun_out/lora/llama_l4.json 2> gpurun_out/lora/llama_l4.err; rc=$?
[ $rc -eq 0 ] || { kill $HB; echo "llama rc=$rc"; tail -5 gpurun_out/lora/llama_l4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/lora/llama_l4.json'));print('llama l4', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'])"
bash scripts/profile_bench.sh llama $P; rc=$?
kill $HB
exit $rc
