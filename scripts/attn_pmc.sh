#!/bin/bash
# PMC counters for the attention kernels (separate runs; kernel-trace only, no sys/hip trace).
#   bash scripts/attn_pmc.sh <tag> [all]
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/attnpmc${1:+_$1}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SETS=("SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT")
if [ "$2" = all ]; then
  SETS+=("SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32" "MfmaUtil" "VALUBusy" "OccupancyPercent")
fi
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$ROOT/scripts/attn_bench.py" 3 > "$OUT/p$i.log" 2>&1 || exit $?
done
echo done
