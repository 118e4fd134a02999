# Round 6: one-client step host issue time with autograd's device thread and on the caller thread.
set -o pipefail
O=${1:-gpurun_out/r6g}
mkdir -p $O
timeout -k 10 300 python -u scripts/host_step_timing.py 4 > $O/host_mt1.txt 2> $O/host_mt1.err || exit 1
HOST_TIMING_AUTOGRAD_MT=0 timeout -k 10 300 python -u scripts/host_step_timing.py 4 > $O/host_mt0.txt 2> $O/host_mt0.err || exit 1
