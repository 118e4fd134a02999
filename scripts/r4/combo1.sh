#!/bin/bash
# new kernels' numerics (skinny LoRA products, fused clip) + the 8-rank rehearsal
set -o pipefail
OUT=gpurun_out/r4_combo1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skinny or lora or grad_clip or rmsnorm" > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" $OUT/pytest.log | head -20; exit 1; }
bash scripts/r4/async8.sh
