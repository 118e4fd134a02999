#!/bin/bash
# Round-3 measurement batch: the reference worker grid (server vs serverless at 5/10/20 clients,
# 20 rounds), BASELINE config 2 (server FedAvg BERT-base, 8 clients) and config 4 (BioBERT +
# PageRank/modified-Z update filter + ledger), 10 timed rounds each, on one MI355X.
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 900 python -u benchmarks/worker_grid.py --out gpurun_out/r3g/worker_grid.json > gpurun_out/r3g/grid.log 2>&1 || { echo "grid rc=$?"; tail -20 gpurun_out/r3g/grid.log; exit 1; }
tail -6 gpurun_out/r3g/grid.log | cut -c1-260
timeout -k 10 300 python -u bench.py --preset baseline2_learnable --mode server --steps 10 --warmup 3 > gpurun_out/r3g/config2.json 2> gpurun_out/r3g/config2.err || { echo "config2 rc=$?"; tail -20 gpurun_out/r3g/config2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3g/config2.json'));print('config2', round(d['value'],4), d['final_accuracy'])"
timeout -k 10 300 python -u bench.py --preset baseline4_learnable --model biobert --steps 10 --warmup 3 > gpurun_out/r3g/config4.json 2> gpurun_out/r3g/config4.err || { echo "config4 rc=$?"; tail -20 gpurun_out/r3g/config4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3g/config4.json'));print('config4', round(d['value'],4), d['final_accuracy'])"
