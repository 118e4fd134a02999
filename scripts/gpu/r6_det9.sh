# Round 6: LayerNorm backward row sums on DPP + v_readlane instead of ds_bpermute (MODE 3):
# numerics against the fp32 reference, then the 4-lane stress test (twice) and MODE 0 control.
set -o pipefail
O=${1:-gpurun_out/r6q}
mkdir -p $O
BCFL_LN_BWD_MODE=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bdaln or layernorm or emb" > $O/numerics.log 2>&1 || exit 1
export DET_MODEL=bert-base
BCFL_LN_BWD_MODE=3 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode3a.jsonl 2> $O/mode3a.err || exit 1
BCFL_LN_BWD_MODE=3 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode3b.jsonl 2> $O/mode3b.err || exit 1
BCFL_LN_BWD_MODE=0 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/mode0.jsonl 2> $O/mode0.err || exit 1
