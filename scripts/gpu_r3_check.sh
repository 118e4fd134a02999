#!/bin/bash
# Round-3 GPU check: kernel + federation GPU tests, then the 8-client and 1-client benches.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_federation.py > gpurun_out/r3/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r3/pytest.log; exit 1; }
tail -3 gpurun_out/r3/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3/bench8.json 2> gpurun_out/r3/bench8.err || { echo "bench8 rc=$?"; tail -20 gpurun_out/r3/bench8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3/bench8.json'));print('8-lane', d['value'], d['final_accuracy'], d['last_round_phases_s'])"
timeout -k 10 300 python -u bench.py --clients 1 --steps 10 --warmup 3 > gpurun_out/r3/bench1.json 2> gpurun_out/r3/bench1.err || { echo "bench1 rc=$?"; tail -20 gpurun_out/r3/bench1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3/bench1.json'));print('1-client', d['value'], d['final_accuracy'])"
