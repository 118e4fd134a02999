#!/bin/bash
# accuracy sweep on the GPU box: scripts/gpu_sweep.sh TAG PRESET ROUNDS COMMON_JSON RUNS_JSON
set -o pipefail
mkdir -p gpurun_out/$1
timeout -k 10 1000 python -u benchmarks/accuracy_curves.py --preset "$2" --rounds "$3" --common "$4" \
  --runs "$5" --out gpurun_out/$1/sweep.json > gpurun_out/$1/sweep.log 2>&1 || { tail -20 gpurun_out/$1/sweep.log; exit 1; }
grep '^{' gpurun_out/$1/sweep.log
