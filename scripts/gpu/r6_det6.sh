# Round 6: LayerNorm backward on fixed inputs under concurrency; the training-step stress test
# with the residual taps (accumulate-into-C dgrad) off.
set -o pipefail
O=${1:-gpurun_out/r6n}
mkdir -p $O
timeout -k 10 200 python -u scripts/ln_bwd_determinism.py 300 > $O/ln_fixed.jsonl 2> $O/ln_fixed.err || exit 1
MODE=acc timeout -k 10 200 python -u scripts/ln_bwd_determinism.py 300 > $O/ln_acc.jsonl 2> $O/ln_acc.err || exit 1
DET_MODEL=bert-base BCFL_RESIDUAL_TAP=0 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/notap.jsonl 2> $O/notap.err || exit 1
