# Round 6: host-blocking calls per round of the one-client layout (cProfile callers).
set -o pipefail
O=${1:-gpurun_out/r6host2}
mkdir -p $O
timeout -k 10 300 python -u scripts/host_step_timing.py 4 > $O/host.txt 2> $O/host.err || exit 1
