set -o pipefail
bash scripts/gpu/r6_cfg4.sh gpurun_out/r6cfg4b || exit 1
bash scripts/gpu/r6_server_grid.sh gpurun_out/r6grid || exit 1
