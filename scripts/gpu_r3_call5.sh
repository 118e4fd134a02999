#!/bin/bash
# worker grid (server vs serverless at 5 / 10 / 20 clients, 20 rounds) after the lanes' local
# evaluation; attention PMC counters (VALU : MFMA) on the LDS-DMA pipeline kernels
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 900 python -u benchmarks/worker_grid.py --out gpurun_out/r3g/worker_grid.json > gpurun_out/r3g/grid.log 2>&1 || { echo "grid rc=$?"; tail -20 gpurun_out/r3g/grid.log; exit 1; }
tail -6 gpurun_out/r3g/grid.log | cut -c1-200
bash scripts/attn_pmc.sh r3 all && python3 scripts/pmc_summary.py gpurun_out/attnpmc_r3 attn > gpurun_out/attnpmc_r3/summary.txt && head -60 gpurun_out/attnpmc_r3/summary.txt
