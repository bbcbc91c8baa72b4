#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_c3_sweep.sh r4c3 &&
bash tools/rehearse_r4.sh
