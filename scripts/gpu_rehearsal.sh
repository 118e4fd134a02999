#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo for the collectives, hipIpc mailboxes between the rank
# processes): the bench JSON at 2 and 4 ranks (device-time phases per rank, info passing over the
# mailbox transport: sync vs async, before / after PageRank removal, analytical prediction), then
# a kernel trace of the one-client-per-rank 2-process run for the device idle-gap timeline.
set -o pipefail
OUT=gpurun_out/rehearsal
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 6 --warmup 2 > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -30 $OUT/n$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/n$n.json'));print('$n', round(d['value'],4), d['final_accuracy'], d['info_passing'] is not None)"
done
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 2 --clients 2 --global-test-samples 250 --steps 8 --warmup 2 --no-info-passing \
  > "$ROOT/$OUT/c2.json" 2> "$ROOT/$OUT/c2.err" || { echo "c2 rc=$?"; tail -30 "$ROOT/$OUT/c2.err"; exit 1; }
python3 "$ROOT/scripts/busy_union.py" $(find "$ROOT/$OUT/prof" -name '*kernel_trace.csv') > "$ROOT/$OUT/c2_busy.json"
find "$ROOT/$OUT/prof" -name '*kernel_trace.csv' | xargs -I{} sh -c 'python3 '"$ROOT"'/scripts/busy_union.py {} > {}.busy.json'
find "$ROOT/$OUT/prof" -name '*kernel_trace.csv' -delete
cat "$ROOT/$OUT/c2_busy.json"
