# usage: bash scripts/gpu/async_sweep_tmp.sh VARIANTS_FILE OUT.jsonl [extra args]
set -o pipefail
cd $GRAFT_REPO_ROOT
VF=$1; OUT=$2; shift 2
args=()
while IFS= read -r line; do [ -n "$line" ] && args+=(--variant "$line"); done < "$VF"
timeout -k 10 1000 python -u benchmarks/async_protocol.py --out $OUT "${args[@]}" "$@" 2>&1 | grep -v Warning
