#!/bin/bash
# 8-rank rehearsal with fresh AdamW again (speed + learning), and its same-round baseline
set -o pipefail
export OUT=gpurun_out/r4_mr4
bash scripts/gpu/rehearse_multirank.sh 8 n8_fresh || exit 1
bash scripts/gpu/rehearse_multirank.sh 8 n8_fresh_unbounded --set gossip_max_lead=0
