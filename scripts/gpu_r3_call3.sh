#!/bin/bash
# tail-kernel diagnostic; config 2 (server FedAvg, lanes' concurrent local eval); multi-rank
# rehearsal (2 / 4 ranks on one GPU, info passing, device-gap timeline of 1 client per rank)
set -o pipefail
mkdir -p gpurun_out/taild gpurun_out/c2
BCFL_G8_TAIL_FORCE=0 timeout -k 10 90 python -u scripts/tail_diag.py > gpurun_out/taild/f0.log 2>&1 || { echo "diag0 rc=$?"; tail gpurun_out/taild/f0.log; exit 1; }
BCFL_G8_TAIL_FORCE=1 timeout -k 10 90 python -u scripts/tail_diag.py > gpurun_out/taild/f1.log 2>&1 || { echo "diag1 rc=$?"; tail gpurun_out/taild/f1.log; exit 1; }
grep force gpurun_out/taild/f*.log
OUT=gpurun_out/c2
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 10 --warmup 3 > $OUT/config2.json 2> $OUT/config2.err || { echo "config2 rc=$?"; tail -20 $OUT/config2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config2.json'));print('config2', round(d['value'],4), d['final_accuracy'], d['last_round_phases_s'])"
bash scripts/gpu_rehearsal.sh
