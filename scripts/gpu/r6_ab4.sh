# Round 6: one-client layout with the runtime-pinned 96 weight-gradient slots (new default for one
# lane) vs 64 forced by the environment, 3 interleaved reps; wgrad kernel tests first.
set -o pipefail
O=${1:-gpurun_out/r6ab4}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or linear_autograd" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--clients 1 --global-test-samples 125"
OUT=$O REPS=3 STEPS=20 WARMUP=5 bash scripts/gpu/bench_ab.sh new "$A" old64 "BCFL_G8_WGRAD_SLOTS=64 $A"
