#!/bin/bash
# after the same-round mix fix: GPU mailbox / federation tests, then multi-rank learning (2 and 4
# ranks on one GPU, the driver's bench config, 20 timed + 5 warmup rounds)
set -o pipefail
OUT=gpurun_out/learn2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_mailbox.py tests/test_gpu_federation.py > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export BCFL_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 20 --warmup 5 > $OUT/n$n.json 2> $OUT/n$n.err || { echo "n$n rc=$?"; tail -20 $OUT/n$n.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/n$n.json') if l.startswith('{')][-1])
print('$n', round(d['value'],4), d['final_accuracy'], d['config']['gossip_mix'], d['multi_rank']['per_rank'][0]['stale_rounds'][-3:])"
done
