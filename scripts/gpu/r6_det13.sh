# Round 6: LayerNorm backward with plain global loads (MODE 8) under the 4-lane stress test; numerics.
set -o pipefail
O=${1:-gpurun_out/r6v}
mkdir -p $O
BCFL_LN_BWD_MODE=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bdaln or emb" > $O/numerics.log 2>&1 || exit 1
export DET_MODEL=bert-base
BCFL_LN_BWD_MODE=8 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode8a.jsonl 2> $O/mode8a.err || exit 1
BCFL_LN_BWD_MODE=8 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode8b.jsonl 2> $O/mode8b.err || exit 1
