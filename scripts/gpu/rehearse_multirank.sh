#!/bin/bash
# N ranks as processes sharing ONE GPU (gloo collectives, hipIpc mailboxes): the bench's multi-rank
# path with accuracy, staleness and wait statistics per rank.
#   bash scripts/gpu/rehearse_multirank.sh N TAG [extra bench.py args, e.g. --set gossip_max_lead=0]
set -o pipefail
N=${1:?ranks}; TAG=${2:?tag}; shift 2
OUT=${OUT:-gpurun_out/multirank}
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
timeout -k 10 450 python -u bench.py --gpus $N --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-info-passing "$@" \
  > $OUT/$TAG.json 2> $OUT/$TAG.err || { echo "$TAG rc=$?"; tail -20 $OUT/$TAG.err; exit 1; }
python3 - $OUT/$TAG.json $TAG <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pr = d.get("multi_rank", {}).get("per_rank", [])
print(sys.argv[2], "s/round", round(d["value"], 4), "final", d["final_accuracy"], "curve", d["accuracy_curve"])
st = lambda p: [x for x in (p.get("stale_rounds") or []) if x is not None]  # noqa: E731
print("  stale mean", [round(sum(st(p)) / max(1, len(st(p))), 2) for p in pr],
      "wait s", [round(p.get("wait_s_total") or 0.0, 2) for p in pr], "lead wait s",
      [round(p.get("lead_wait_s_total") or 0.0, 2) for p in pr])
PY
