# Round 6: kernel determinism under concurrency (fixed batch + dropout keys per replica, L
# concurrent streams, every iteration must reproduce every gradient bit), then 20 more lanes runs.
set -o pipefail
O=${1:-gpurun_out/r6i}
mkdir -p $O
timeout -k 10 300 python -u scripts/kernel_determinism.py 150 3 > $O/det_2l_l3.jsonl 2> $O/det_2l_l3.err || exit 1
timeout -k 10 300 python -u scripts/kernel_determinism.py 100 3 --overlap-wgrad > $O/det_2l_l3_ovl.jsonl 2> $O/det_2l_l3_ovl.err || exit 1
DET_MODEL=bert-base timeout -k 10 400 python -u scripts/kernel_determinism.py 40 4 --overlap-wgrad > $O/det_base_l4_ovl.jsonl 2> $O/det_base_l4_ovl.err || exit 1
timeout -k 10 400 python -u scripts/lanes_repro.py 20 3 > $O/repro_l3.jsonl 2> $O/repro_l3.err || exit 1
