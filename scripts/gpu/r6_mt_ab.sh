# Round 6: backward on the caller thread (default) vs autograd's device thread, interleaved A/B of
# the one-client layout and the driver config, host step timing, and a kernel trace of the
# one-client bench for the device-gap census.
set -o pipefail
O=${1:-gpurun_out/r6h}
mkdir -p $O
timeout -k 10 200 python -u scripts/host_step_timing.py 4 > $O/host_caller.txt 2> $O/host_caller.err || exit 1
OUT=$O/ab1 REPS=2 STEPS=20 WARMUP=5 timeout -k 10 900 bash scripts/gpu/bench_ab.sh \
  caller "--clients 1 --global-test-samples 125" thread "BCFL_AUTOGRAD_THREAD=1 --clients 1 --global-test-samples 125" > $O/ab1.txt 2>&1 || exit 1
OUT=$O/ab8 REPS=2 STEPS=10 WARMUP=3 timeout -k 10 900 bash scripts/gpu/bench_ab.sh \
  caller "" thread "BCFL_AUTOGRAD_THREAD=1" > $O/ab8.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof1 -o p1 -- python bench.py --steps 10 --warmup 3 --clients 1 --global-test-samples 125 > $O/prof1.log 2>&1 || exit 1
