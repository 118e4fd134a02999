# Round 6: weight-gradient slot fine-tuning — one-client layout 80 / 96 / 112, driver config 64 / 96.
set -o pipefail
O=${1:-gpurun_out/r6ab5}
A="--clients 1 --global-test-samples 125"
OUT=$O/one REPS=2 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  s80 "BCFL_G8_WGRAD_SLOTS=80 $A" s96 "$A" s112 "BCFL_G8_WGRAD_SLOTS=112 $A" || exit 1
OUT=$O/eight REPS=2 STEPS=10 WARMUP=3 bash scripts/gpu/bench_ab.sh s64 "" s96 "BCFL_G8_WGRAD_SLOTS=96"
