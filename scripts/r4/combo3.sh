#!/bin/bash
# SwiGLU-epilogue numerics -> config-5 record + profile; IID sweep 2; copy census
set -o pipefail
bash scripts/r4/cfg5.sh || exit 1
bash scripts/r4/iid2.sh || exit 1
bash scripts/r4/copies.sh
