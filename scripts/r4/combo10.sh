#!/bin/bash
# async rehearsals after the pacing fix (8 ranks: defaults / fresh AdamW; 4 ranks), the config-2
# record with the IID protocol, the copy trace and the skinny grid sweep
set -o pipefail
OUT=gpurun_out/r4_mr2 bash scripts/gpu/rehearse_multirank.sh 8 n8 || exit 1
OUT=gpurun_out/r4_mr2 bash scripts/gpu/rehearse_multirank.sh 8 n8_fresh_adamw --set async_keep_optimizer_state=false || exit 1
OUT=gpurun_out/r4_mr2 bash scripts/gpu/rehearse_multirank.sh 4 n4 || exit 1
mkdir -p gpurun_out/r4_cfg2
timeout -k 10 400 python -u bench.py --preset baseline2_learnable --mode server --steps 20 --warmup 5 > gpurun_out/r4_cfg2/bench.json 2> gpurun_out/r4_cfg2/bench.err || { echo "cfg2 rc=$?"; tail -5 gpurun_out/r4_cfg2/bench.err; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r4_cfg2/bench.json') if l.startswith('{')][-1])
print('cfg2', round(d['value'],4), d['final_accuracy'], d['accuracy_curve'])"
OUT=gpurun_out/r4_copies2 bash scripts/gpu/copy_trace.sh || exit 1
OUT=gpurun_out/r4_skinny bash scripts/skinny_sweep.sh
