#!/bin/bash
set -o pipefail
bash scripts/gpu_r3_learn.sh || exit 1
bash scripts/gpu_r3_callB.sh
