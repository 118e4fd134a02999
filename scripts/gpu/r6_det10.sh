# Round 6: LayerNorm backward with an agent-scope acquire at kernel start (MODE 4) and with
# system-coherent input loads (MODE 5), 4-lane stress test each (twice for MODE 4).
set -o pipefail
O=${1:-gpurun_out/r6r}
mkdir -p $O
export DET_MODEL=bert-base
BCFL_LN_BWD_MODE=4 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode4a.jsonl 2> $O/mode4a.err || exit 1
BCFL_LN_BWD_MODE=5 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode5.jsonl 2> $O/mode5.err || exit 1
BCFL_LN_BWD_MODE=4 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode4b.jsonl 2> $O/mode4b.err || exit 1
