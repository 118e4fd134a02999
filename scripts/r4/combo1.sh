#!/bin/bash
# new kernels' numerics (skinny LoRA products, fused clip) + the 8-rank rehearsal
set -o pipefail
OUT=gpurun_out/r4_combo1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skinny or lora or grad_clip or rmsnorm" > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 240 python -u scripts/copy_census.py --clients 1 --rounds 2 > $OUT/census_1client.txt 2>&1 || { echo "census rc=$?"; tail -20 $OUT/census_1client.txt; exit 1; }
head -30 $OUT/census_1client.txt
bash scripts/r4/async8.sh
