#!/bin/bash
# what the driver runs at round end, in one call: the GPU suite, smoke(), the N = 1 bench
set -o pipefail
OUT=${OUT:-gpurun_out/final_check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 180 --timeout-method thread tests > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('metric','value','unit','ms_per_step','final_accuracy','vs_baseline')})"
