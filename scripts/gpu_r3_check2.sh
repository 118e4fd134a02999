#!/bin/bash
# Round-3 GPU check 2: federation/ckpt GPU tests, then benches (8 lanes; 1 client with the full
# draw; 1 client with a 1/8 draw = the per-rank eval work of the 8-GPU layout).
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_federation.py tests/test_gpu_ckpt.py > gpurun_out/r3b/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r3b/pytest.log; exit 1; }
tail -2 gpurun_out/r3b/pytest.log
for cfg in "8:--steps 10 --warmup 3" "1:--clients 1 --steps 10 --warmup 3" "1e:--clients 1 --global-test-samples 125 --steps 10 --warmup 3"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/r3b/bench$tag.json 2> gpurun_out/r3b/bench$tag.err || { echo "bench$tag rc=$?"; tail -20 gpurun_out/r3b/bench$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3b/bench$tag.json'));print('$tag', round(d['value'],4), d['final_accuracy'], 'dev/wall', round(d['device_span_vs_wall'] or 0,3), {k:round(v,4) for k,v in d['timed_rounds_device_phases_mean_s'].items()})"
done
