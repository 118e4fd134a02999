# Round 6 closing measurements on the final tree: GPU suite, smoke(), the N = 1 driver bench and
# the one-client layout (20 timed + 5 warm-up rounds each), rocprofv3 kernel stats of the latter.
set -o pipefail
O=${1:-gpurun_out/r6final2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 180 --timeout-method thread tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench8.json 2> $O/bench8.err || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --clients 1 --global-test-samples 125 > $O/bench1.json 2> $O/bench1.err || exit 1
bash scripts/profile_bench.sh r6f2_1 --clients 1 --global-test-samples 125 > $O/prof1.log 2>&1 || exit 1
