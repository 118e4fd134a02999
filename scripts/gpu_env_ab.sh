#!/bin/bash
# A/B the bench under environment settings, interleaved twice:
#   scripts/gpu_env_ab.sh TAG "VAR=a" "VAR=b" ...   ("-" = no extra variable)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  i=0
  for e in "$@"; do
    if [ "$e" = "-" ]; then envs=(); else envs=($e); fi
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/$TAG/b${rep}_$i.log 2>&1 \
      || { echo "bench [$e] failed"; tail -20 gpurun_out/$TAG/b${rep}_$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/b${rep}_$i.log').read().strip().splitlines()[-1]); print('[$e]', round(d['value'],4), 's/round', round(d['last_round_phases_s'].get('t_train'),4))"
    i=$((i+1))
  done
done
