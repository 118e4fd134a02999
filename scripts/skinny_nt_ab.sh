#!/bin/bash
# skinny.hip: non-temporal streaming loads of the big operand on / off, 2 interleaved reps
set -o pipefail
OUT=${OUT:-gpurun_out/skinny_nt}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skinny or lora" > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for nt in 2 1; do
    BCFL_SKINNY_NT=$nt timeout -k 10 120 python -u scripts/lora_mlp_bench.py 8192 --skinny-only > $OUT/nt${nt}_$rep.jsonl 2>&1 || { echo "nt$nt rc=$?"; exit 1; }
    python3 -c "
import json
rs=[json.loads(l) for l in open('$OUT/nt${nt}_$rep.jsonl') if l.startswith('{')]
print('nt $nt rep $rep', [(r['op'][7:], r.get('K') or r.get('N'), r['R'], round(r['us'],1)) for r in rs], round(sum(r['us'] for r in rs),1))"
  done
done
