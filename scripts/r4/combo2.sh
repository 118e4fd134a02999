#!/bin/bash
# 8-rank rehearsal with the bounded-lead default, then the IID learning sweep
set -o pipefail
bash scripts/r4/async8.sh || exit 1
bash scripts/r4/iid_sweep.sh
