# Round 6: LayerNorm kernels built without packed-fp32 VALU ops, 4-lane stress test (MODE 0).
set -o pipefail
O=${1:-gpurun_out/r6y}
mkdir -p $O
export DET_MODEL=bert-base
timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/nopk_a.jsonl 2> $O/nopk_a.err || exit 1
timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/nopk_b.jsonl 2> $O/nopk_b.err || exit 1
