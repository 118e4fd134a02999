# Round 6: one-client layout, evaluation results read through pinned copies on the evaluation
# stream vs .cpu() at resolve time (BCFL_EVAL_READ_SYNC=1: synchronises the training stream).
set -o pipefail
A="--clients 1 --global-test-samples 125"
OUT=${1:-gpurun_out/r6ab8} REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh \
  pinned "$A" sync "BCFL_EVAL_READ_SYNC=1 $A" && \
  timeout -k 10 300 python -u scripts/host_block_probe.py --clients 1 --global-test-samples 125 --steps 6 --warmup 2 > gpurun_out/r6ab8/hbp.json 2> gpurun_out/r6ab8/hbp.err
