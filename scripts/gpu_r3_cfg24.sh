#!/bin/bash
# BASELINE configs 2 and 4 on the final tree (6 default lanes), 10 timed + 3 warmup rounds
set -o pipefail
OUT=gpurun_out/cfg24
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 10 --warmup 3 > $OUT/config2.json 2> $OUT/config2.err || { echo "config2 rc=$?"; tail -20 $OUT/config2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config2.json'));print('config2', round(d['value'],4), d['final_accuracy'], d['config']['client_lanes_per_gpu'])"
timeout -k 10 300 python -u bench.py --preset baseline4_learnable --model biobert --steps 10 --warmup 3 > $OUT/config4.json 2> $OUT/config4.err || { echo "config4 rc=$?"; tail -20 $OUT/config4.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config4.json'));print('config4', round(d['value'],4), d['final_accuracy'], d['config']['client_lanes_per_gpu'])"
