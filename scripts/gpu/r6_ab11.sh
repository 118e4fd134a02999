# Round 6: one-client layout after the round-start local-score read became non-blocking; eval
# forwards replayed from hipGraphs vs eager.
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab11} REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  graphs "$A" eager "BCFL_EVAL_GRAPHS=0 $A"
