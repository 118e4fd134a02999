# Round 6: LayerNorm backward row-pipeline variants under the 4-lane stress test.
set -o pipefail
O=${1:-gpurun_out/r6p}
mkdir -p $O
export DET_MODEL=bert-base
BCFL_LN_BWD_MODE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode1.jsonl 2> $O/mode1.err || exit 1
BCFL_LN_BWD_MODE=2 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode2.jsonl 2> $O/mode2.err || exit 1
BCFL_LN_BWD_MODE=0 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode0.jsonl 2> $O/mode0.err || exit 1
