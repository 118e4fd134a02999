# Round 6: 3-lane / 1-lane cross-run reproducibility (first divergence located), the same under the
# stream race checker, then config 2 and one worker-grid rep with the gated hold-out selection.
set -o pipefail
O=${1:-gpurun_out/r6d}
mkdir -p $O
timeout -k 10 300 python -u scripts/lanes_repro.py 12 3 > $O/repro_l3.jsonl 2> $O/repro_l3.err || exit 1
timeout -k 10 300 python -u scripts/lanes_repro.py 10 1 > $O/repro_l1.jsonl 2> $O/repro_l1.err || exit 1
BCFL_DEBUG_STREAMS=1 timeout -k 10 400 python -u scripts/lanes_repro.py 2 3 > $O/repro_l3_dbg.jsonl 2> $O/repro_l3_dbg.err || exit 1
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 20 --warmup 5 --out runs/cfg2 > $O/cfg2.json 2> $O/cfg2.err || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid.json > $O/grid.log 2>&1 || exit 1
