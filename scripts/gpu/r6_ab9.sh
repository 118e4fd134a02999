# Round 6: one-client layout, local-evaluation forwards issued after the round's exchange and the
# global-evaluation snapshot on the training stream (default) vs the local evaluation issued
# right after its snapshot (BCFL_EVAL_LOCAL_EARLY=1) and vs both round-end reads synchronous.
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab9} REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  late "$A" early "BCFL_EVAL_LOCAL_EARLY=1 $A" early_sync "BCFL_EVAL_LOCAL_EARLY=1 BCFL_EVAL_READ_SYNC=1 $A"
