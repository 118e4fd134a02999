#!/bin/bash
# 4-rank async learning variance: defaults x2, fresh AdamW x2, the same-round barrier
set -o pipefail
export OUT=gpurun_out/r4_mr3
bash scripts/gpu/rehearse_multirank.sh 4 n4_a || exit 1
bash scripts/gpu/rehearse_multirank.sh 4 n4_fresh_a --set async_keep_optimizer_state=false || exit 1
bash scripts/gpu/rehearse_multirank.sh 4 n4_b || exit 1
bash scripts/gpu/rehearse_multirank.sh 4 n4_fresh_b --set async_keep_optimizer_state=false || exit 1
bash scripts/gpu/rehearse_multirank.sh 4 n4_same --set drift_same_round_mix=true || exit 1
bash scripts/gpu/rehearse_multirank.sh 8 n8_final
