# Round 6: LayerNorm backward inputs (dout, z, mean, rstd, gamma) before and after the kernel.
set -o pipefail
O=${1:-gpurun_out/r6s}
mkdir -p $O
DET_MODEL=bert-base DET_PROBE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 30 4 > $O/probe.jsonl 2> $O/probe.err || exit 1
