#!/bin/bash
# The final round-4 artifacts on the cut-skipping tree (tools/run_round4.sh), then the
# four-rank rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/run_round4.sh r4final2 &&
bash tools/rehearse_r4_n4.sh
