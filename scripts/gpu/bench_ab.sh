#!/bin/bash
# Interleaved A/B of bench.py variants on one GPU: each variant is one bench run (STEPS timed +
# WARMUP warm-up rounds), REPS interleaved repetitions; prints s/round, final accuracy and the
# mean device phases per variant.
#   bash scripts/gpu/bench_ab.sh TAG1 "ARGS1" TAG2 "VAR=value ARGS2" ...
set -o pipefail
OUT=${OUT:-gpurun_out/bench_ab}
mkdir -p $OUT
REPS=${REPS:-1}
for rep in $(seq 1 $REPS); do
  set -- "${@}"
  args=("$@")
  i=0
  while [ $i -lt ${#args[@]} ]; do
    tag=${args[$i]}; a=${args[$((i + 1))]}; i=$((i + 2))
    # leading VAR=value words of a variant are its environment
    envs=(); rest=()
    for w in $a; do
      if [ ${#rest[@]} -eq 0 ] && [[ $w == *=* ]] && [[ $w != --* ]]; then envs+=("$w"); else rest+=("$w"); fi
    done
    # shellcheck disable=SC2086
    env "${envs[@]}" timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} "${rest[@]}" \
      > $OUT/${tag}_r$rep.json 2> $OUT/${tag}_r$rep.err || { echo "$tag rc=$?"; tail -20 $OUT/${tag}_r$rep.err; exit 1; }
    python3 - $OUT/${tag}_r$rep.json $tag $rep <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d.get("timed_rounds_device_phases_mean_s", {})
print(sys.argv[2], "rep", sys.argv[3], round(d["value"], 4), d["final_accuracy"],
      {k: round(v, 4) for k, v in ph.items() if k in ("dev_t_train", "dev_t_comm", "dev_t_round", "dev_t_eval_global")},
      flush=True)
PY
  done
done
