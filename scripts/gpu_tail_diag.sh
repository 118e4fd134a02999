#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/taild
BCFL_G8_TAIL_FORCE=0 timeout -k 10 90 python -u scripts/tail_diag.py 2>&1 | tee gpurun_out/taild/f0.log && \
BCFL_G8_TAIL_FORCE=1 timeout -k 10 90 python -u scripts/tail_diag.py 2>&1 | tee gpurun_out/taild/f1.log
