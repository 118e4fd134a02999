#!/bin/bash
# skinny.hip grid-size sweep at the config-5 shapes (one process per setting: the targets are read
# once per process)
set -o pipefail
OUT=${OUT:-gpurun_out/skinny_sweep}
mkdir -p $OUT
for xw in 2048 4096 8192; do
  for pw in 512 1024 2048 4096; do
    BCFL_SKINNY_XWT_WAVES=$xw BCFL_SKINNY_PTX_WGS=$pw timeout -k 10 120 python -u scripts/lora_mlp_bench.py 8192 --skinny-only > $OUT/x${xw}_p${pw}.jsonl 2>&1 || { echo "x$xw p$pw rc=$?"; tail -3 $OUT/x${xw}_p${pw}.jsonl; exit 1; }
    python3 -c "
import json
rs=[json.loads(l) for l in open('$OUT/x${xw}_p${pw}.jsonl') if l.startswith('{')]
print('xwt $xw ptx $pw', [(r['op'][7:], r.get('K') or r.get('N'), r['R'], round(r['us'],1)) for r in rs], round(sum(r['us'] for r in rs),1))"
  done
done
