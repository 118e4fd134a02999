# Round 6: cross-lane nondeterminism — which op's backward output first differs (gradient trace).
set -o pipefail
O=${1:-gpurun_out/r6m}
mkdir -p $O
export DET_MODEL=bert-base
DET_TRACE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/trace.jsonl 2> $O/trace.err || exit 1
DET_TRACE=1 timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/trace2.jsonl 2> $O/trace2.err || exit 1
