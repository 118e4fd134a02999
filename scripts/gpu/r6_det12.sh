# Round 6: producer-side L2 writeback (accumulate GEMM release fence), consumer acquire + coherent
# loads together, and the LayerNorm backward with its block order reversed.
set -o pipefail
O=${1:-gpurun_out/r6u}
mkdir -p $O
export DET_MODEL=bert-base
BCFL_G8_ACC_FENCE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/accfence.jsonl 2> $O/accfence.err || exit 1
BCFL_LN_BWD_MODE=6 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode6.jsonl 2> $O/mode6.err || exit 1
BCFL_LN_BWD_MODE=7 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode7.jsonl 2> $O/mode7.err || exit 1
