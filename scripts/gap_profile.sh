#!/bin/bash
# Device idle gaps over a bench run (kernel trace only): where does the GPU wait for the host?
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/gaps
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 6 --warmup 2 "$@" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
t=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/scripts/busy_union.py" "$t" > "$OUT/busy.json"
rm -rf "$OUT/prof"
cat "$OUT/busy.json"
