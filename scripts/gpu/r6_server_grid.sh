# Server-mode stability (hold-out selection) and the serverless-vs-server worker grid, round 6.
set -o pipefail
O=${1:-gpurun_out/r6grid}
mkdir -p $O
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 20 --warmup 5 --out runs/cfg2 > $O/cfg2.json 2> $O/cfg2.err || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep1.json > $O/grid_rep1.log 2>&1 || exit 1
