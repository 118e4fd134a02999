#!/bin/bash
# Round-3 GPU check 3: mailbox (side-stream fetch, info passing), federation (server lanes),
# then the 8-lane bench.
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_mailbox.py tests/test_gpu_federation.py > gpurun_out/r3c/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r3c/pytest.log; exit 1; }
grep -E "passed|failed|\{'sync'" gpurun_out/r3c/pytest.log | tail -4
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3c/bench8.json 2> gpurun_out/r3c/bench8.err || { echo "bench8 rc=$?"; tail -20 gpurun_out/r3c/bench8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3c/bench8.json'));print('8', round(d['value'],4), d['final_accuracy'], round(d['device_span_vs_wall'],3))"
