#!/bin/bash
# LoRA on split-K 8-phase skinny GEMMs + tail segments: numerics, config 5; attention PMC
set -o pipefail
mkdir -p gpurun_out/lora
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lora or rmsnorm or llama or rope or swiglu" > gpurun_out/lora/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/lora/pytest.log; exit 1; }
tail -2 gpurun_out/lora/pytest.log
( while sleep 30; do echo "hb $(date +%s)" >> gpurun_out/lora/hb.log; done ) & HB=$!
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 400 python -u bench.py $P --steps 5 --warmup 1 > gpurun_out/lora/llama_g8.json 2> gpurun_out/lora/llama_g8.err; rc=$?
kill $HB
[ $rc -eq 0 ] || { echo "llama rc=$rc"; tail -5 gpurun_out/lora/llama_g8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/lora/llama_g8.json'));print('llama g8', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'], d['final_train_loss'])"
bash scripts/attn_pmc.sh r3 all && python3 scripts/pmc_summary.py gpurun_out/attnpmc_r3 attn > gpurun_out/attnpmc_r3/summary.txt && head -50 gpurun_out/attnpmc_r3/summary.txt
