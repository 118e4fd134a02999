# Round 6: LayerNorm backward probe with value samples; every lane the same batch shape (different
# weights) so a differing value can be compared with the other lanes' outputs.
set -o pipefail
O=${1:-gpurun_out/r6w}
mkdir -p $O
DET_MODEL=bert-base DET_PROBE=1 DET_SAME_BATCH=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 30 4 > $O/probe.jsonl 2> $O/probe.err || exit 1
