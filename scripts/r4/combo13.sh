#!/bin/bash
# full GPU suite on the final tree, then the config-5 record + profile (vectorized RoPE, skinny grid)
set -o pipefail
OUT=gpurun_out/r4_final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 180 --timeout-method thread tests > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit 1; }
OUT=gpurun_out/r4_cfg5b STEPS=8 bash scripts/gpu/config5.sh
