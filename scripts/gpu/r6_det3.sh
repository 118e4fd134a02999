# Round 6: bisect the cross-lane nondeterminism (bert-base, 4 lanes, no side-stream wgrad):
# serialised lanes, persistent GEMM grids off, reference attention / LayerNorm / GEMM paths.
set -o pipefail
O=${1:-gpurun_out/r6k}
mkdir -p $O
export DET_MODEL=bert-base
DET_SERIAL=1 timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/serial.jsonl 2> $O/serial.err || exit 1
timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/base.jsonl 2> $O/base.err || exit 1
BCFL_G8_PERSIST=0 timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/nopersist.jsonl 2> $O/nopersist.err || exit 1
BCFL_TORCH_OPS=gemm,gemm_act timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/torchgemm.jsonl 2> $O/torchgemm.err || exit 1
BCFL_TORCH_OPS=bdaln,emb_ln timeout -k 10 200 python -u scripts/kernel_determinism.py 40 4 > $O/torchln.jsonl 2> $O/torchln.err || exit 1
BCFL_TORCH_OPS=attn,subset_attn timeout -k 10 300 python -u scripts/kernel_determinism.py 20 4 > $O/torchattn.jsonl 2> $O/torchattn.err || exit 1
