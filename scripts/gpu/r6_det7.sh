# Round 6: LayerNorm backward inputs / outputs at kernel time across iterations (4 lanes), and the
# stress test with one hardware queue per lane stream.
set -o pipefail
O=${1:-gpurun_out/r6o}
mkdir -p $O
export DET_MODEL=bert-base
DET_PROBE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 30 4 > $O/probe.jsonl 2> $O/probe.err || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/hwq8.jsonl 2> $O/hwq8.err || exit 1
