#!/bin/bash
# Round-3 re-entry check: the driver's 1-GPU bench and the one-client round, then config 5 A/B.
set -o pipefail
OUT=gpurun_out/r3r
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench8.json 2> $OUT/bench8.err || { echo "bench8 rc=$?"; tail -20 $OUT/bench8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench8.json'));print('8', round(d['value'],4), d['final_accuracy'])"
timeout -k 10 300 python -u bench.py --clients 1 --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench1 rc=$?"; tail -20 $OUT/bench1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench1.json'));print('1', round(d['value'],4), d['final_accuracy'])"
bash scripts/gpu_llama_ab.sh
