#!/bin/bash
# A/B the bench under op routings: scripts/gpu_ab.sh TAG "ROUTING1" "ROUTING2" ... (BCFL_TORCH_OPS values)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for r in "$@"; do
  BCFL_TORCH_OPS="$r" timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/$TAG/b$i.log 2>&1 || { echo "bench [$r] failed"; tail -20 gpurun_out/$TAG/b$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$TAG/b$i.log').read().strip().splitlines()[-1]); print('[$r]', round(d['value'],4), 's/round', d['last_round_phases_s'].get('t_train'))"
  i=$((i+1))
done
