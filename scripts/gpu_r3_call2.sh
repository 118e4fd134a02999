#!/bin/bash
# config 2 (server FedAvg, lanes' concurrent local eval), the multi-rank rehearsal, then a kernel
# summary of the config-5 round (Llama-3-8B LoRA, local batch 32).
set -o pipefail
OUT=gpurun_out/c2
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 10 --warmup 3 > $OUT/config2.json 2> $OUT/config2.err || { echo "config2 rc=$?"; tail -20 $OUT/config2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config2.json'));print('config2', round(d['value'],4), d['final_accuracy'], d['last_round_phases_s'])"
bash scripts/gpu_rehearsal.sh || exit 1
bash scripts/profile_bench.sh llama --model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100 --batch-size 32
