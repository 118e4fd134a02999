#!/bin/bash
# overlapped weight gradient vs inline, persistent 8-phase grids off / on
set -o pipefail
mkdir -p gpurun_out/ovl
for v in 0 1; do
  BCFL_G8_PERSIST=$v timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "overlapped_wgrad" > gpurun_out/ovl/p$v.log 2>&1; echo "persist=$v rc=$?"
  grep -E "passed|failed" gpurun_out/ovl/p$v.log | tail -1
done
