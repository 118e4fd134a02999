#!/bin/bash
# kernel summaries of the final round-3 tree: the driver's 8-lane round and the one-client round
set -o pipefail
bash scripts/profile_bench.sh final8 && bash scripts/profile_bench.sh final1 --clients 1 --global-test-samples 125
