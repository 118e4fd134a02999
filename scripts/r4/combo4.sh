#!/bin/bash
# LoRA MLP / skinny microbench, full GPU suite, the bounded-lead 8-rank rehearsal, information
# passing at 2 / 4 processes
set -o pipefail
OUT=gpurun_out/r4_gputest
mkdir -p $OUT
timeout -k 10 240 python -u scripts/lora_mlp_bench.py 8192 > $OUT/lora_mlp_bench.jsonl 2>&1 || { echo "mlp bench rc=$?"; tail -5 $OUT/lora_mlp_bench.jsonl; exit 1; }
cat $OUT/lora_mlp_bench.jsonl | grep '^{'
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 180 --timeout-method thread tests > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; [ $rc -eq 1 ] || exit 1; }
bash scripts/r4/async8.sh || exit 1
bash scripts/r4/infopass.sh
