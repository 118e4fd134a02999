# Round 6: GPU suite on the split tree, server hold-out (selection + optimizer rollback) on
# config 2 and the worker grid (2 interleaved reps, server and serverless), and the 3-lane
# cross-run reproducibility check (ROADMAP #8).
set -o pipefail
O=${1:-gpurun_out/r6c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 20 --warmup 5 --out runs/cfg2 > $O/cfg2.json 2> $O/cfg2.err || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep1.json > $O/grid_rep1.log 2>&1 || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep2.json > $O/grid_rep2.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/lanes_repro.py 15 > $O/lanes_repro.jsonl 2> $O/lanes_repro.err || exit 1
