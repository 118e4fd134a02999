#!/bin/bash
# where the one-client round's runtime copy kernels come from: torch.profiler op chains, then a
# rocprofv3 kernel + memory-copy trace (stats only)
set -o pipefail
OUT=gpurun_out/r4_copies
mkdir -p $OUT
timeout -k 10 240 python -u scripts/copy_census.py --clients 1 --rounds 2 --torch-prof > $OUT/ops.txt 2>&1 || { echo "census rc=$?"; tail -20 $OUT/ops.txt; exit 1; }
head -45 $OUT/ops.txt
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --clients 1 --global-test-samples 125 --steps 2 --warmup 1 > "$ROOT/$OUT/prof.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
for f in $(find "$ROOT/$OUT/prof" -name '*memory_copy_stats.csv'); do echo "== $f"; cat "$f"; done
MC=$(find "$ROOT/$OUT/prof" -name '*memory_copy_trace.csv' | head -1)
[ -n "$MC" ] && python3 - "$MC" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print("memory_copy_trace columns:", list(rows[0].keys()) if rows else None)
c = collections.Counter(); t = collections.Counter()
for r in rows:
    k = (r.get("Direction"), r.get("Size") or r.get("Bytes") or r.get("Copy_Bytes"))
    c[k] += 1; t[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, n in c.most_common(30):
    print(k, n, round(t[k] / n / 1e3, 1), "us avg")
PY
STATS=$(find "$ROOT/$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/scripts/summarize_prof.py" "$STATS" > "$ROOT/$OUT/summary.md"
find "$ROOT/$OUT/prof" -name '*_trace.csv' -delete
head -40 "$ROOT/$OUT/summary.md"
