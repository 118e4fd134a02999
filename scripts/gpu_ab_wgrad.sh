#!/bin/bash
# A/B of the weight-gradient kernel inside the full bench: K9 (gemm.hip) vs the 8-phase kernel
# (gemm8.hip) at 128 / 256 slots; 8 lanes and 1 client, interleaved, one box.
set -o pipefail
mkdir -p gpurun_out/abw
for rep in 1 2; do
for v in "k9:BCFL_WGRAD_G8=0" "g8s128:BCFL_WGRAD_G8=1 BCFL_G8_WGRAD_SLOTS=128" "g8s256:BCFL_WGRAD_G8=1 BCFL_G8_WGRAD_SLOTS=256"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-ckpt > gpurun_out/abw/${tag}_8_$rep.json 2>/dev/null || { echo "fail $tag"; exit 1; }
  env $envs timeout -k 10 200 python -u bench.py --clients 1 --global-test-samples 125 --steps 8 --warmup 2 --no-ckpt > gpurun_out/abw/${tag}_1_$rep.json 2>/dev/null || { echo "fail1 $tag"; exit 1; }
  python -c "import json;a=json.load(open('gpurun_out/abw/${tag}_8_$rep.json'));b=json.load(open('gpurun_out/abw/${tag}_1_$rep.json'));print('$tag rep$rep 8-lane', round(a['value'],4), '1-client', round(b['value'],4))"
done
done
