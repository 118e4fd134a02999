#!/bin/bash
# LoRA tail-segment GEMM numerics + config 5 with it; config 2 (server FedAvg, lanes' concurrent
# local eval); the multi-rank rehearsal; then a kernel summary of the config-5 round.
set -o pipefail
OUT=gpurun_out/c2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lora or g8 or linear" > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
P="--model llama3-8b-lora --preset baseline5_llama3_8b_lora_serverless --global-test-samples 100"
timeout -k 10 420 python -u bench.py $P --steps 3 --warmup 1 > $OUT/llama.json 2> $OUT/llama.err || { echo "llama rc=$?"; tail -20 $OUT/llama.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/llama.json'));print('llama', round(d['value'],3), d['tokens_per_s'], d['hbm_peak_gb'], d['config'])"
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 10 --warmup 3 > $OUT/config2.json 2> $OUT/config2.err || { echo "config2 rc=$?"; tail -20 $OUT/config2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config2.json'));print('config2', round(d['value'],4), d['final_accuracy'], d['last_round_phases_s'])"
bash scripts/gpu_rehearsal.sh || exit 1
bash scripts/profile_bench.sh llama $P
