# Round 6: one-client layout, persistent GEMM grids on / 256-row tiles pinned, vs default (96 slots).
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab6} REPS=2 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  base "$A" persist "BCFL_G8_PERSIST=1 $A" bm256 "BCFL_G8_BM=256 $A"
