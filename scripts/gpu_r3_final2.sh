#!/bin/bash
# after the dy / dres aliasing fix: overlap diagnosis, the two failing tests, then the full suite
set -o pipefail
OUT=gpurun_out/final2
mkdir -p $OUT
timeout -k 10 120 python -u scripts/overlap_diag.py > $OUT/ovl.log 2>&1 || { echo "diag rc=$?"; tail -5 $OUT/ovl.log; exit 1; }
grep overlap= $OUT/ovl.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfEX --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -8 $OUT/pytest.log
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
