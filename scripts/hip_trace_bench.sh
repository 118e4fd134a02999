#!/bin/bash
# HIP runtime API + kernel trace of a short bench run (no PMC): launch-vs-execution lag analysis.
# Only the small summary stays under gpurun_out/ (the raw traces exceed the copy-back limit).
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
RAW=/tmp/hiptrace_bench
OUT=$ROOT/gpurun_out/hiptrace_bench
mkdir -p "$OUT" "$RAW"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace -d "$RAW" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 > "$OUT/log.txt" 2>&1 || exit $?
python3 "$ROOT/scripts/launch_lag.py" "$RAW" > "$OUT/summary.txt" 2>&1
cp "$RAW/lag_summary.json" "$OUT/" 2>/dev/null
ls -la "$RAW" >> "$OUT/summary.txt"
