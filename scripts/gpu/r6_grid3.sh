# Round 6: host issue vs device time of the one-client step, then two worker-grid reps with the
# serverless global model scored as the reference does (the mean of the client models, once).
set -o pipefail
O=${1:-gpurun_out/r6f}
mkdir -p $O
timeout -k 10 300 python -u scripts/host_step_timing.py 4 > $O/host_timing.txt 2> $O/host_timing.err || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep1.json > $O/grid_rep1.log 2>&1 || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep2.json > $O/grid_rep2.log 2>&1 || exit 1
