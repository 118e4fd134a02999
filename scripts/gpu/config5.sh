#!/bin/bash
# config 5 (Llama-3-8B LoRA, 8 clients): LoRA kernel numerics, a K-round record, a kernel profile
#   STEPS=10 bash scripts/gpu/config5.sh
set -o pipefail
OUT=${OUT:-gpurun_out/config5}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lora or skinny or rmsnorm or swiglu or pack" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py --preset baseline5_llama3_8b_lora_serverless --model llama3-8b-lora --steps ${STEPS:-8} --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('cfg5', round(d['value'],3), d['final_accuracy'], d['final_majority_rate'], d['global_eval_rows'], d['accuracy_curve'])"
[ -n "$NO_PROF" ] && exit 0
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --preset baseline5_llama3_8b_lora_serverless --model llama3-8b-lora --steps 1 --warmup 1 > "$ROOT/$OUT/prof.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
STATS=$(find "$ROOT/$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/scripts/summarize_prof.py" "$STATS" > "$ROOT/$OUT/summary.md"
find "$ROOT/$OUT/prof" -name '*kernel_trace.csv' -delete
head -30 "$ROOT/$OUT/summary.md"
