#!/bin/bash
# after the dy / dres aliasing fix: overlap diagnosis, the two failing tests, then the full suite
set -o pipefail
OUT=gpurun_out/final4
mkdir -p $OUT
timeout -k 10 120 python -u scripts/overlap_diag.py > $OUT/ovl.log 2>&1 || { echo "diag rc=$?"; tail -5 $OUT/ovl.log; exit 1; }
grep overlap= $OUT/ovl.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfEX --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -8 $OUT/pytest.log
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench8.json 2> $OUT/bench8.err || { echo "bench8 rc=$?"; tail -20 $OUT/bench8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench8.json'));print('8', round(d['value'],4), d['final_accuracy'], round(d['device_span_vs_wall'],3))"
timeout -k 10 300 python -u bench.py --clients 1 --global-test-samples 125 --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench1 rc=$?"; tail -20 $OUT/bench1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench1.json'));print('1', round(d['value'],4), d['final_accuracy'])"
