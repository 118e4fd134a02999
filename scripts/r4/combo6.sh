#!/bin/bash
# where the one-client round's runtime copies come from; skinny grid sweep; weight-gradient slots A/B
set -o pipefail
bash scripts/r4/copies2.sh || exit 1
OUT=gpurun_out/r4_skinny bash scripts/skinny_sweep.sh || exit 1
bash scripts/r4/slots_ab.sh
