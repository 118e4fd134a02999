#!/bin/bash
# 8-rank rehearsal with the final async defaults; IID protocol + worker grid
set -o pipefail
bash scripts/r4/async8.sh || exit 1
mkdir -p gpurun_out/r4_iidfinal
timeout -k 10 900 python -u scripts/iid_protocol.py --out gpurun_out/r4_iidfinal/iid_final.json --scratch gpurun_out/r4_iidfinal/tmp.json > gpurun_out/r4_iidfinal/log.txt 2>&1; rc=$?
grep '^{' gpurun_out/r4_iidfinal/log.txt
exit $rc
