#!/bin/bash
# PMC counters for the linear.hip kernels (separate passes, kernel trace only).
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/linpmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  PYTHONPATH=$ROOT timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$ROOT/scripts/linear_pmc_bench.py" 2 > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" linear > "$OUT/summary.txt"
rm -rf "$OUT"/p*/
cat "$OUT/summary.txt"
