#!/bin/bash
# kernel-trace stats + PMC counters for the K9 wgrad kernel (separate runs, no sys/hip trace)
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/gemmpmc${1:+_$1}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$ROOT/scripts/gemm_bench.py" 10 > "$OUT/stats.log" 2>&1 || exit $?
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$ROOT/scripts/gemm_bench.py" 2 > "$OUT/p$i.log" 2>&1 || exit $?
done
echo done
