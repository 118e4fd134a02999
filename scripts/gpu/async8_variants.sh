#!/bin/bash
# 8 ranks sharing ONE GPU (the driver's 8-GPU layout, time-sliced): which async-gossip settings keep
# the label-sharded federation learning. Each variant is one bench.py run (25 rounds); the summary
# line per variant: s/round, final accuracy, curve, mean staleness and lead waits per rank.
#   bash scripts/gpu/async8_variants.sh TAG1 "ARGS1" TAG2 "ARGS2" ...
set -o pipefail
OUT=${OUT:-gpurun_out/async8_variants}
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
while [ $# -ge 2 ]; do
  tag=$1; args=$2; shift 2
  # shellcheck disable=SC2086
  timeout -k 10 300 python -u bench.py --gpus ${GPUS:-8} --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
    --no-info-passing $args > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -20 $OUT/$tag.err; exit 1; }
  python3 - $OUT/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pr = d.get("multi_rank", {}).get("per_rank", [])
print(sys.argv[2], round(d["value"], 3), d["final_accuracy"], d["accuracy_curve"], flush=True)
print("   stale", [round(sum(p["stale_rounds"]) / max(1, len(p["stale_rounds"])), 2) for p in pr],
      "lead wait", [round(p.get("lead_wait_s_total", 0), 2) for p in pr], flush=True)
PY
done
