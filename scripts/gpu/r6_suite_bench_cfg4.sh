set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench8.json 2> $O/bench8.err || exit 1
timeout -k 10 400 python -u bench.py --preset baseline4_learnable --model biobert --steps 20 --warmup 5 --set 'inject_byzantine={"3": 50.0}' --out runs/cfg4 > $O/cfg4.json 2> $O/cfg4.err || exit 1
cp runs/cfg4/metrics.jsonl $O/cfg4_metrics.jsonl
grep -c verdict runs/cfg4/ledger.jsonl > $O/cfg4_verdict_blocks.txt || true
