set -o pipefail
mkdir -p gpurun_out/acc
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k adamw -x -q --timeout 120 --timeout-method thread > gpurun_out/acc/pytest.log 2>&1 || { tail -20 gpurun_out/acc/pytest.log; exit 1; }
tail -2 gpurun_out/acc/pytest.log
timeout -k 10 600 python -u benchmarks/accuracy_curves.py --preset baseline3_learnable --rounds 25 --out gpurun_out/acc/curves.json > gpurun_out/acc/curves.log 2>&1 || { tail -20 gpurun_out/acc/curves.log; exit 1; }
tail -4 gpurun_out/acc/curves.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/acc/bench.log 2>&1 || { tail -20 gpurun_out/acc/bench.log; exit 1; }
tail -1 gpurun_out/acc/bench.log
