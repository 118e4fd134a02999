#!/bin/bash
# round-4 start: GPU suite, smoke and the driver bench on the round-3 tree
set -o pipefail
OUT=gpurun_out/r4_sanity
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfEX --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -4 $OUT/pytest.log
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value'],4), d['final_accuracy'], round(d['device_span_vs_wall'],3))"
