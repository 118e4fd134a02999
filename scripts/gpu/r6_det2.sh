# Round 6: which switch makes the lanes path nondeterministic — caller-thread backward vs autograd's
# worker thread, side-stream weight gradients on / off, one lane vs four.
set -o pipefail
O=${1:-gpurun_out/r6j}
mkdir -p $O
BCFL_AUTOGRAD_THREAD=1 timeout -k 10 300 python -u scripts/lanes_repro.py 10 3 > $O/repro_l3_thread.jsonl 2> $O/repro_l3_thread.err || exit 1
BCFL_AUTOGRAD_THREAD=1 DET_MODEL=bert-base timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 --overlap-wgrad > $O/det_base_l4_ovl_thread.jsonl 2> $O/det_base_l4_ovl_thread.err || exit 1
DET_MODEL=bert-base timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/det_base_l4_noovl.jsonl 2> $O/det_base_l4_noovl.err || exit 1
DET_MODEL=bert-base timeout -k 10 300 python -u scripts/kernel_determinism.py 60 1 --overlap-wgrad > $O/det_base_l1_ovl.jsonl 2> $O/det_base_l1_ovl.err || exit 1
