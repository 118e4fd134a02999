# Round 6: one-client layout, weight-gradient tile slots 64 (default) / 96 / 128, 3 interleaved reps.
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab3} REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  base "$A" slots96 "BCFL_G8_WGRAD_SLOTS=96 $A" slots128 "BCFL_G8_WGRAD_SLOTS=128 $A"
