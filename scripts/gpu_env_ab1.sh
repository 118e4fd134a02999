#!/bin/bash
# A/B a 1-client bench (the per-rank work of an 8-GPU run) under environment settings, twice.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  i=0
  for e in "$@"; do
    if [ "$e" = "-" ]; then envs=(); else envs=($e); fi
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --clients 1 --steps 8 --warmup 3 > gpurun_out/$TAG/c${rep}_$i.log 2>&1 \
      || { echo "bench [$e] failed"; tail -20 gpurun_out/$TAG/c${rep}_$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/c${rep}_$i.log').read().strip().splitlines()[-1]); print('1-client [$e]', round(d['value'],4), 's/round')"
    i=$((i+1))
  done
done
