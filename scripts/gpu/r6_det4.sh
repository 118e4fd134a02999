# Round 6: cross-lane nondeterminism, continued: saved-activation check, LayerNorm vs embedding
# kernels separately, reference attention over 40 iterations.
set -o pipefail
O=${1:-gpurun_out/r6l}
mkdir -p $O
export DET_MODEL=bert-base
DET_SAVED=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 30 4 > $O/saved.jsonl 2> $O/saved.err || exit 1
BCFL_TORCH_OPS=bdaln timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/torch_bdaln.jsonl 2> $O/torch_bdaln.err || exit 1
BCFL_TORCH_OPS=emb_ln timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/torch_embln.jsonl 2> $O/torch_embln.err || exit 1
BCFL_TORCH_OPS=attn,subset_attn timeout -k 10 400 python -u scripts/kernel_determinism.py 40 4 > $O/torch_attn.jsonl 2> $O/torch_attn.err || exit 1
