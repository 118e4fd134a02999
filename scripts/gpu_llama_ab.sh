#!/bin/bash
# Config 5 (Llama-3-8B LoRA, 8 clients on one GPU): local batch 32 (the reference's batch, ~8k
# tokens per GEMM) with auto lanes and one lane; then a kernel summary of the batch-32 round.
set -o pipefail
OUT=gpurun_out/llama
mkdir -p $OUT
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 420 python -u bench.py $P --batch-size 32 --steps 3 --warmup 1 > $OUT/b32.json 2> $OUT/b32.err || { echo "b32 rc=$?"; tail -20 $OUT/b32.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/b32.json'));print('b32', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'], d['config']['client_lanes_per_gpu'])"
timeout -k 10 420 python -u bench.py $P --batch-size 32 --lanes 1 --steps 3 --warmup 1 > $OUT/b32l1.json 2> $OUT/b32l1.err || { echo "b32l1 rc=$?"; tail -20 $OUT/b32l1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/b32l1.json'));print('b32l1', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'], d['config']['client_lanes_per_gpu'])"
