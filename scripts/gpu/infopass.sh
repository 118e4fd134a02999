#!/bin/bash
# information passing (plain + BC-FL, all three detectors) at N processes sharing one GPU
#   bash scripts/gpu/infopass.sh 2 4
set -o pipefail
OUT=${OUT:-gpurun_out/infopass}
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
for n in "$@"; do
  timeout -k 10 300 python -u bench.py --gpus $n --steps 4 --warmup 2 > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -20 $OUT/n$n.err; exit 1; }
  python3 - $OUT/n$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
from bcfl.trust.infopass import summary
print("world", d["n_gpus"], "p2p median GB/s", round((d.get("p2p_post_measured") or {}).get("gb_per_s_median", 0), 1))
for line in summary(d.get("info_passing") or {}):
    print(" ", line)
PY
done
