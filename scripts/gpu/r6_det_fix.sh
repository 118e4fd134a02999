# Round 6: the LayerNorm kernels built without packed-fp32 VALU ops — LN numerics, the 4-lane stress
# test with and without side-stream weight gradients, the 2-layer 3-lane overlap case, and 20
# three-lane federation runs (lanes_repro, 19 / 20 differing before the fix).
set -o pipefail
O=${1:-gpurun_out/r6z}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bdaln or emb" > $O/numerics.log 2>&1 || exit 1
DET_MODEL=bert-base timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 > $O/det_base_l4.jsonl 2> $O/det_base_l4.err || exit 1
DET_MODEL=bert-base timeout -k 10 300 python -u scripts/kernel_determinism.py 40 4 --overlap-wgrad > $O/det_base_l4_ovl.jsonl 2> $O/det_base_l4_ovl.err || exit 1
timeout -k 10 300 python -u scripts/kernel_determinism.py 100 3 --overlap-wgrad > $O/det_2l_l3_ovl.jsonl 2> $O/det_2l_l3_ovl.err || exit 1
timeout -k 10 400 python -u scripts/lanes_repro.py 20 3 > $O/repro_l3.jsonl 2> $O/repro_l3.err || exit 1
