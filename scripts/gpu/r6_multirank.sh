# Round 6: the multi-rank bench path on the final tree, ranks as processes sharing one GPU (gloo
# collectives, hipIpc mailboxes): N = 2 / 4 serverless, N = 2 server, N = 8 on equal 32-CU slices.
set -o pipefail
export OUT=${1:-gpurun_out/r6mr}
[ -n "$ONLY_N8" ] || { STEPS=10 WARMUP=3 bash scripts/gpu/rehearse_multirank.sh 2 n2 || exit 1; }
[ -n "$ONLY_N8" ] || { STEPS=10 WARMUP=3 bash scripts/gpu/rehearse_multirank.sh 4 n4 || exit 1; }
[ -n "$ONLY_N8" ] || { STEPS=10 WARMUP=3 bash scripts/gpu/rehearse_multirank.sh 2 n2_server --mode server || exit 1; }
BCFL_REHEARSE_CUS=256 STEPS=10 WARMUP=3 bash scripts/gpu/rehearse_multirank.sh 8 n8_cu || exit 1
