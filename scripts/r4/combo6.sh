#!/bin/bash
# where the one-client round's runtime copies come from; weight-gradient slot budget A/B
set -o pipefail
bash scripts/r4/copies2.sh || exit 1
bash scripts/r4/slots_ab.sh
