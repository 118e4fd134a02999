# Round 6: two interleaved worker-grid reps (server vs serverless at 5 / 10 / 20 clients) after the
# serverless global-model score moved its snapshot onto the training stream; GPU federation tests first.
set -o pipefail
O=${1:-gpurun_out/r6e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_federation.py -m gpu > $O/gpufed.log 2>&1 || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep1.json > $O/grid_rep1.log 2>&1 || exit 1
timeout -k 10 900 python -u benchmarks/worker_grid.py --clients 5 10 20 --rounds 20 --out $O/grid_rep2.json > $O/grid_rep2.log 2>&1 || exit 1
