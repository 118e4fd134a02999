# BASELINE config 4 (BioBERT, label-shard clients, async round-complete gossip, PageRank + mod-Z
# update filter inside the application, ledger), one Byzantine client (client 4, updates boosted
# 50x); 20 timed rounds after 5 warm-up rounds, N = 1. CLIENTS: 8 (the BASELINE shape: 3 vs 4
# honest clients per class after the rejection) or 9 (8 honest + 1).
set -o pipefail
O=${1:-gpurun_out/r6cfg4}
mkdir -p $O
timeout -k 10 400 python -u bench.py --preset baseline4_learnable --model biobert --clients ${CLIENTS:-8} --steps 20 --warmup 5 --set 'inject_byzantine={"4": 50.0}' --out runs/cfg4 > $O/cfg4.json 2> $O/cfg4.err || exit 1
cp runs/cfg4/metrics.jsonl $O/cfg4_metrics.jsonl
timeout -k 10 400 python -u bench.py --preset baseline4_learnable --model biobert --clients ${CLIENTS:-8} --steps 20 --warmup 5 --set 'inject_byzantine={"4": 50.0}' --set filter_redistribute='"uniform"' --out runs/cfg4u > $O/cfg4_uniform.json 2> $O/cfg4_uniform.err || exit 1
