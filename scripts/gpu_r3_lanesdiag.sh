#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/lanesdiag
for i in 1 2 3; do timeout -k 10 240 python -u scripts/lanes_diag2.py 1 >> gpurun_out/lanesdiag/d.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/lanesdiag/d.log; exit 1; }; done
grep wgrad= gpurun_out/lanesdiag/d.log | cut -c1-250
