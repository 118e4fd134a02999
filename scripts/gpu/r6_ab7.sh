# Round 6: one-client layout, device-resident update roots read by the deferred ledger vs the
# round-end host reads (BCFL_ROUND_SYNC=1: roots, loss sum and ledger read inside the round).
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab7} REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  deferred "$A" sync "BCFL_ROUND_SYNC=1 $A"
