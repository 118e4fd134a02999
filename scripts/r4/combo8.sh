#!/bin/bash
# full GPU suite; one-client + driver benches (overlapped optimizer A/B); 8-rank rehearsal with the
# round-4 async defaults; config-5 record
set -o pipefail
OUT=gpurun_out/r4_onec
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 180 --timeout-method thread tests > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; [ $rc -eq 1 ] || exit 1; }
timeout -k 10 300 python -u bench.py --clients 1 --global-test-samples 125 --steps 20 --warmup 3 > $OUT/b1.json 2> $OUT/b1.err || { echo "b1 rc=$?"; tail -5 $OUT/b1.err; exit 1; }
timeout -k 10 300 python -u bench.py --clients 1 --global-test-samples 125 --steps 20 --warmup 3 --set overlap_optimizer=false > $OUT/b1_noopt.json 2> $OUT/b1_noopt.err || { echo "b1n rc=$?"; tail -5 $OUT/b1_noopt.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/b8.json 2> $OUT/b8.err || { echo "b8 rc=$?"; tail -5 $OUT/b8.err; exit 1; }
python3 - <<'PY'
import json
for t in ("b1", "b1_noopt", "b8"):
    d = json.loads([l for l in open(f"gpurun_out/r4_onec/{t}.json") if l.startswith("{")][-1])
    print(t, round(d["value"], 4), d["final_accuracy"], d.get("device_span_vs_wall"),
          {k: round(v, 4) for k, v in d["timed_rounds_device_phases_mean_s"].items()})
PY
bash scripts/r4/async8.sh || exit 1
bash scripts/r4/cfg5.sh
