# Round 6: one-client layout GEMM knobs — all GEMMs on 128-row tiles, 96 / 48 weight-gradient slots.
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab2} REPS=2 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  base "$A" bm128 "BCFL_G8_BM=128 $A" slots96 "BCFL_G8_WGRAD_SLOTS=96 $A" slots48 "BCFL_G8_WGRAD_SLOTS=48 $A"
