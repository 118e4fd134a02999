#!/bin/bash
# final check + the 2-rank async rehearsal on the same tree
set -o pipefail
bash scripts/gpu/final_check.sh || exit 1
OUT=gpurun_out/final_mr bash scripts/gpu/rehearse_multirank.sh 2 n2_final
