#!/bin/bash
# GPU-box check: kernel/federation tests, a 1-GPU bench run and a rocprofv3 kernel profile of it.
# Usage: scripts/gpu_check.sh TAG [bench args...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-chk}; shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 "$@" > "$OUT/bench.log" 2>&1 \
  || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 2 "$@" > "$OUT/prof_bench.log" 2>&1 \
  || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof_bench.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/scripts/summarize_prof.py" "$f" "bench $TAG" > "$OUT/kernel_stats.md"
cp "$f" "$OUT/kernel_stats.csv"
t=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
[ -n "$t" ] && python3 "$ROOT/scripts/busy_union.py" "$t" > "$OUT/busy.json"
rm -rf "$OUT/prof"  # full traces exceed gpurun's 64 MiB copy-back
head -30 "$OUT/kernel_stats.md"
