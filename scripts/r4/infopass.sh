#!/bin/bash
# information passing (plain + BC-FL, all three detectors) measured at 2 and 4 processes on one GPU
set -o pipefail
OUT=gpurun_out/r4_infopass
mkdir -p $OUT
export BCFL_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $n --steps 4 --warmup 2 > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -20 $OUT/n$n.err; exit 1; }
  python - $OUT/n$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
ip, pp = d.get("info_passing") or {}, d.get("p2p_post_measured") or {}
print("world", d["n_gpus"], "p2p median GB/s", round(pp.get("gb_per_s_median", 0), 1))
bw = ip.get("bw_MBps")
if bw:
    print("infopass bw GB/s", [[round(x / 1e3, 1) for x in row] for row in bw])
for s in ip.get("sources", []):
    print(" src", s["source"], "sync", round(s["measured_sync_s"] * 1e3, 3), "async", round(s["measured_async_s"] * 1e3, 3),
          "bcfl", round(s["bcfl"]["sync_s"] * 1e3, 3), round(s["bcfl"]["async_s"] * 1e3, 3))
for det, e in (ip.get("detectors") or {}).items():
    print(" ", det, e["flagged"], len(e["sources"]))
PY
done
