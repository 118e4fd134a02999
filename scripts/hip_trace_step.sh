#!/bin/bash
# HIP runtime API trace of a few training steps (no PMC): find blocking API calls
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/hiptrace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$ROOT/scripts/step_cpu_vs_gpu.py" > "$OUT/log.txt" 2>&1
