#!/bin/bash
# the one-client round's runtime copy kernels attributed to their neighbouring kernels
set -o pipefail
OUT=${OUT:-gpurun_out/copy_trace}
mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --clients 1 --global-test-samples 125 --steps 2 --warmup 1 > "$ROOT/$OUT/prof.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
KT=$(find "$ROOT/$OUT/prof" -name '*kernel_trace.csv' | head -1)
head -1 "$KT" > "$ROOT/$OUT/columns.txt"
python3 "$ROOT/scripts/copy_neighbors.py" "$KT" > "$ROOT/$OUT/neighbors.txt"
find "$ROOT/$OUT/prof" -name '*_trace.csv' -delete
cat "$ROOT/$OUT/columns.txt"; head -45 "$ROOT/$OUT/neighbors.txt"
