# Round-5 default asynchronous protocol: 1-GPU bench (in-process virtual ranks) + 8 ranks on equal
# 32-CU slices of one MI355X (the pacing of 8 GPUs), N runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r5proto; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench rc=$?"; tail -20 $OUT/bench_n1.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_n1.json') if l.startswith('{')][-1])
print('n1', round(d['value'],4), d['final_accuracy'], d['accuracy_curve'], d['config']['protocol'])"
export BCFL_REHEARSE_CUS=256
OUT=$OUT bash scripts/gpu/async8_variants.sh ${RUNS:-cu8_a "" cu8_b "" cu8_c "" cu8_d "" cu8_e ""}
