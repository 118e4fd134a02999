#!/bin/bash
# kernel-trace stats + PMC counters of the 8-phase weight-gradient (and forward) GEMMs at the bench
# shapes: separate runs, one counter set each, kernel trace only (no sys / hip trace)
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/gemmpmc${1:+_$1}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$ROOT/scripts/gemm_bench.py" 10 fwd > "$OUT/stats.log" 2>&1 || exit $?
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$ROOT/scripts/gemm_bench.py" 2 fwd > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" g8_kernel > "$OUT/pmc_summary.txt" 2>&1
STATS=$(find "$OUT/stats" -name '*kernel_stats.csv' | head -1)
[ -n "$STATS" ] && python3 "$ROOT/scripts/summarize_prof.py" "$STATS" > "$OUT/summary.md"
find "$OUT" -name '*kernel_trace.csv' -size +20M -delete
echo done
