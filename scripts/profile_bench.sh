#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (writes gpurun_out/prof/*).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof${1:+_$1}
shift || true
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 "$@" > "$OUT/bench.log" 2>&1
tail -3 "$OUT/bench.log"
# keep the stats, drop the per-dispatch trace (tens of MB: gpurun copies back <= 64 MiB)
STATS=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
[ -n "$STATS" ] && python3 "$ROOT/scripts/summarize_prof.py" "$STATS" > "$OUT/summary.md"
find "$OUT" -name '*kernel_trace.csv' -delete
find "$OUT" -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'head -30 {}'
