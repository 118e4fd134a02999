#!/bin/bash
# Final-tree check: which gradients the overlapped weight gradient changes (persistent grids off /
# on), full GPU suite, smoke(), the driver's 1-GPU bench (20 timed + 5 warmup) and the one-client
# round (the per-rank work of the 8-GPU layout).
set -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
for v in 0 1; do
  BCFL_G8_PERSIST=$v timeout -k 10 120 python -u scripts/overlap_diag.py > $OUT/ovl_p$v.log 2>&1 || { echo "diag rc=$?"; tail -5 $OUT/ovl_p$v.log; exit 1; }
  echo "persist=$v"; grep overlap= $OUT/ovl_p$v.log | cut -c1-220
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfEX --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -12 $OUT/pytest.log
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench8.json 2> $OUT/bench8.err || { echo "bench8 rc=$?"; tail -20 $OUT/bench8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench8.json'));print('8', round(d['value'],4), d['final_accuracy'], round(d['device_span_vs_wall'],3))"
timeout -k 10 300 python -u bench.py --clients 1 --global-test-samples 125 --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench1 rc=$?"; tail -20 $OUT/bench1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench1.json'));print('1', round(d['value'],4), d['final_accuracy'])"
