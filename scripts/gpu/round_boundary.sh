#!/bin/bash
# the one-client round boundary on the device (kernel trace of a short one-client bench)
set -o pipefail
OUT=${OUT:-gpurun_out/round_boundary}
mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --clients 1 --global-test-samples 125 --steps 4 --warmup 1 > "$ROOT/$OUT/prof.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
KT=$(find "$ROOT/$OUT/prof" -name '*kernel_trace.csv' | head -1)
head -1 "$KT" > "$ROOT/$OUT/columns.txt"
python3 "$ROOT/scripts/round_boundary.py" "$KT" > "$ROOT/$OUT/boundary.txt"
find "$ROOT/$OUT/prof" -name '*_trace.csv' -delete
tail -5 "$ROOT/$OUT/boundary.txt"
