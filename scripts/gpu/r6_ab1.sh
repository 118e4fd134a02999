# Round 6: one-client layout A/B on the final tree — default vs backward-overlapped AdamW vs two
# concurrent micro-batches (2 interleaved reps, 20 timed + 5 warm-up rounds).
set -o pipefail
OUT=${1:-gpurun_out/r6ab1} REPS=2 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  base "--clients 1 --global-test-samples 125" \
  ovlopt "--clients 1 --global-test-samples 125 --set overlap_optimizer=true" \
  micro2 "--clients 1 --global-test-samples 125 --micro-batches 2"
