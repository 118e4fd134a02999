# Round 6: LayerNorm backward without the IEEE division sequence for the row means (MODE 9).
set -o pipefail
O=${1:-gpurun_out/r6x}
mkdir -p $O
export DET_MODEL=bert-base
BCFL_LN_BWD_MODE=9 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode9a.jsonl 2> $O/mode9a.err || exit 1
BCFL_LN_BWD_MODE=9 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode9b.jsonl 2> $O/mode9b.err || exit 1
